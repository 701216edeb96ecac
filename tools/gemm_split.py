"""The grouped projection backward vs its parts at the C2 shapes (T = 8192): dX alone (esgpt_gemm_bf16), dW alone
(esgpt_linear_bwd without dx: split-K plan for the whole chip), and the grouped pair (esgpt_linear_bwd)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_bwd, linear_dx  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402


def main():
    T = int(os.environ.get("T", 8192))
    for out, inn in [(768, 256), (256, 256), (1024, 256), (256, 1024), (1624, 256)]:
        x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * out * inn
        tdx = gtime(lambda: linear_dx(dy, w))
        tdw = gtime(lambda: linear_bwd(dy, x, w, need_dx=False, need_db=True))
        tp = gtime(lambda: linear_bwd(dy, x, w, need_db=True))
        print(f"({out},{inn}) dX {tdx:6.1f}us {fl / tdx / 1e6:5.0f}TF | dW+db {tdw:6.1f}us {fl / tdw / 1e6:5.0f}TF | "
              f"pair {tp:6.1f}us {2 * fl / tp / 1e6:5.0f}TF", flush=True)


if __name__ == "__main__":
    main()
