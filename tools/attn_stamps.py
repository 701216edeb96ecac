"""In-kernel s_memtime stamps of the attention backward: the library built with -DESGPT_STAMPS as
eventstreamgpt_amd/libesgpt_amd_stamps.so (tools/build_stamps.sh), loaded via ESGPT_AMD_LIB and called through the C
ABI (ctypes). Prints the phase times (memtime ticks, 100 MHz) of one workgroup at the C2 shape, with dropout."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd import _lib as L  # noqa: E402

B, Lq, H, hd = 32, 256, 4, 64
D = H * hd
dev = torch.device("cuda")
lib = L.load()
em = torch.ones(B, Lq, dtype=torch.uint8, device=dev)
qkv = (0.5 * torch.randn(B, Lq, 3 * D, device=dev)).bfloat16()
o = torch.empty(B, Lq, D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, H, Lq, device=dev)
seed = torch.tensor([99], dtype=torch.int64, device=dev)
q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
st = L.stream()
p = 0.1 if len(sys.argv) < 2 else float(sys.argv[1])
L.check(lib.esgpt_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), 3 * D, Lq, o.data_ptr(), D, lse.data_ptr(),
                           em.data_ptr(), em.data_ptr(), B, H, Lq, Lq, hd, 0, p, seed.data_ptr(), L.BF16, st), "fwd")
do = torch.randn(B, Lq, D, device=dev).bfloat16()
dqkv = torch.empty_like(qkv)
nb = lib.esgpt_attn_bwd_workspace(B, H, Lq, Lq, hd)
ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
cnt = torch.zeros(int(lib.esgpt_attn_bwd_counters(B, H, Lq)), dtype=torch.int32, device=dev)
for _ in range(3):
    L.check(lib.esgpt_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), 3 * D, Lq, o.data_ptr(), D, do.data_ptr(), D,
                               lse.data_ptr(), em.data_ptr(), em.data_ptr(), dqkv[..., :D].data_ptr(),
                               dqkv[..., D:2 * D].data_ptr(), dqkv[..., 2 * D:].data_ptr(), 3 * D, B, H, Lq, Lq, hd, 0,
                               p, seed.data_ptr(), L.BF16, ws.data_ptr(), nb, cnt.data_ptr(), st), "bwd")
torch.cuda.synchronize()
buf = (ctypes.c_uint64 * 64)()
lib.esgpt_debug_stamps.argtypes = [ctypes.c_void_p]
lib.esgpt_debug_stamps(buf)
stp = list(buf)
t0 = stp[0]
names = {0: "start", 1: "prologue", 40: "loop end", 41: "dkv stored"}
for i in [0, 1] + list(range(2, 2 + 6 * 4)) + [40, 41]:
    if stp[i]:
        nm = names.get(i, f"tile{(i - 2) // 6}.{['bar1', 'staged', 'computed', 'bar3', 'dq mfma', 'dq stored'][(i - 2) % 6]}")
        print(f"{nm:24s} {stp[i] - t0:8d}", flush=True)
