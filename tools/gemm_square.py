"""A few launches of one large bf16 GEMM (fwd form, both operands K-contiguous) for counter passes:
    rocprofv3 --pmc <counters> -- python tools/gemm_square.py [S] [N] [K]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_fwd  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N = int(sys.argv[2]) if len(sys.argv) > 2 else M
K = int(sys.argv[3]) if len(sys.argv) > 3 else M
x = torch.rand(M, K, device="cuda").mul_(2).sub_(1).bfloat16()
w = torch.rand(N, K, device="cuda").mul_(2).sub_(1).bfloat16()
for _ in range(5):
    y = linear_fwd(x, w)
torch.cuda.synchronize()
print("ok", float(y.float().abs().mean()))
