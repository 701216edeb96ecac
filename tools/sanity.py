"""Box sanity: large bf16 GEMM rate, HBM copy rate, and the projection GEMM shapes of the C2 step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
us = t(lambda: a @ b, 10)
print(f"mm 8192^3 bf16: {us:.1f} us  {2 * 8192**3 / us / 1e6:.0f} TF/s")
x = torch.empty(2**28, device="cuda", dtype=torch.float32)
y = torch.empty_like(x)
us = t(lambda: y.copy_(x), 10)
print(f"copy 1 GiB: {us:.1f} us  {2 * x.numel() * 4 / us / 1e3:.0f} GB/s")
z = torch.empty(16, device="cuda")
us = t(lambda: z.add_(1), 200)
print(f"tiny kernel back-to-back: {us:.2f} us")
from eventstreamgpt_amd.fused import linear_fwd  # noqa: E402
xa = torch.randn(8192, 256, device="cuda", dtype=torch.bfloat16)
w = torch.randn(768, 256, device="cuda", dtype=torch.bfloat16)
us = t(lambda: linear_fwd(xa, w), 50)
print(f"hip gemm 8192x768x256: {us:.1f} us  {2 * 8192 * 768 * 256 / us / 1e6:.0f} TF/s")
