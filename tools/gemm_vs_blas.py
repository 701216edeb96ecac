"""Our projection GEMMs vs hipBLASLt (torch.matmul, bf16) at the C2 step's shapes: forward y = x·Wᵀ, dX = dY·W and
dW = dYᵀ·X (f32 output for ours; torch's dW is bf16-out, so its time is a lower bound), each timed as 20 launches
in a HIP graph. Prints µs and TFLOP/s per product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_bwd, linear_fwd  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402


def main():
    T = int(os.environ.get("T", 8192))
    for out, inn in [(768, 256), (256, 256), (1024, 256), (256, 1024), (1624, 256)]:
        x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * out * inn
        rows = [("ours fwd", lambda: linear_fwd(x, w), fl),
                ("blas fwd", lambda: x @ w.t(), fl),
                ("ours bwd(dX+dW+db)", lambda: linear_bwd(dy, x, w, need_db=True), 2 * fl),
                ("blas dX", lambda: dy @ w, fl),
                ("blas dW", lambda: dy.t() @ x, fl),
                ("blas dW f32out", lambda: torch.matmul(dy.t().float(), x.float()), fl)]
        line = []
        for name, fn, f in rows:
            us = gtime(fn)
            line.append(f"{name} {us:6.1f}us {f / us / 1e6:5.0f}TF")
        print((out, inn), " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
