"""Runs attention fwd+bwd at one shape a few times (for rocprofv3 kernel timing). argv: B L H hd [window] [p]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.kernels import AttentionFn  # noqa: E402

B, L, H, hd = (int(x) for x in sys.argv[1:5])
window = int(sys.argv[5]) if len(sys.argv) > 5 else 0
p = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
D = H * hd
em = torch.ones(B, L, dtype=torch.bool, device="cuda")
qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda")).bfloat16().requires_grad_(True)
for _ in range(5):
    o = AttentionFn.apply(qkv, em, em, H, window, False, p)
    torch.autograd.grad(o, qkv, torch.randn_like(o))
torch.cuda.synchronize()
print("done")
