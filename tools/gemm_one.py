"""One forward projection shape launched repeatedly (for PMC passes): python tools/gemm_one.py [din dout reps]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_fwd  # noqa: E402

din, dout, reps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (256, 768, 50)))
x = torch.randn(8192, din, device="cuda").bfloat16()
w = (0.05 * torch.randn(dout, din, device="cuda")).bfloat16()
b = torch.randn(dout, device="cuda")
for _ in range(reps):
    linear_fwd(x, w, b)
torch.cuda.synchronize()
