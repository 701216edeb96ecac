"""In-kernel s_memtime stamps of the attention backward (library built with -DESGPT_STAMPS as
libesgpt_amd_stamps.so; load it via ESGPT_AMD_LIB). Prints phase deltas (memtime ticks) of one workgroup."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import AttentionFn  # noqa: E402

B, Lq, H, hd = 32, 256, 4, 64
D = H * hd
em = torch.ones(B, Lq, dtype=torch.bool, device="cuda")
qkv = (0.5 * torch.randn(B, Lq, 3 * D, device="cuda")).bfloat16().requires_grad_(True)
lib = L.load()
for _ in range(3):
    o = AttentionFn.apply(qkv, em, em, H, 0, False, 0.0)
    torch.autograd.grad(o, qkv, torch.randn_like(o))
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * 64)()
lib.esgpt_debug_stamps(buf)
st = list(buf)
t0 = st[0]
names = {0: "start", 1: "prologue", 40: "loop end", 41: "dkv stored"}
for i in [0, 1] + list(range(2, 2 + 6 * 4)) + [40, 41]:
    if st[i]:
        nm = names.get(i, f"tile{(i - 2) // 6}.{['bar1', 'staged', 'computed', 'bar3', 'dq mfma', 'dq stored'][(i - 2) % 6]}")
        print(f"{nm:24s} {st[i] - t0:8d}")
