"""Runs the C2 projection GEMM shapes through the HIP GEMM (fwd, dX, dW) a few times each (for rocprofv3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_dw, linear_dx, linear_fwd  # noqa: E402

N = 8192
for out, inn in [(768, 256), (256, 1024)]:
    x = torch.randn(N, inn, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, out, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        linear_fwd(x, w)
        linear_dx(dy, w)
        linear_dw(dy, x)
torch.cuda.synchronize()
print("done")
