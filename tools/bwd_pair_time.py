"""Graph-timed grouped projection backward (esgpt::linear_bwd: dX + dW + db in one launch) at the C2 step's five
shapes (T = 8192 tokens). Tools build + ESGPT_GEMM_DBG bits isolate its parts (tools/bwd_sweep.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.kernels import tickets  # noqa: E402
from eventstreamgpt_amd import ops as O  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402

O.load()
T = 8192
tot = 0.0
for name, out, inn, act in [("qkv", 768, 256, -1), ("out_proj", 256, 256, -1), ("c_fc", 1024, 256, -1),
                            ("c_proj+gelu'", 256, 1024, 0), ("head", 1624, 256, -1)]:
    x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
    pre = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16) if act >= 0 else None
    tk = tickets(x.device)
    fn = lambda: torch.ops.esgpt.linear_bwd(dy, x, w, None, act, pre, True, True, tk, None, None)  # noqa: E731
    us = gtime(fn)
    tot += us * (1 if name == "head" else 6)
    print(f"{name:13s} {us:7.2f} us  {4 * T * out * inn / us / 1e6:6.1f} TFLOP/s", flush=True)
print(f"step total (6 layers + head): {tot:.1f} us", flush=True)
