import os, sys, ctypes
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd import _lib as L
from eventstreamgpt_amd.fused import linear_dw, linear_dx, linear_fwd
lib = L.load()
lib.esgpt_gemm_debug.argtypes = [ctypes.c_int]
def t(fn, it=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
N = 8192
for out, inn in [(768, 256), (256, 1024)]:
    x = torch.randn(N, inn, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, out, device="cuda", dtype=torch.bfloat16)
    for dbg in (0, 1, 2, 3):
        lib.esgpt_gemm_debug(dbg)
        print((out, inn), "dbg", dbg, " ".join(f"{k} {t(f):6.1f}us" for k, f in
              [("fwd", lambda: linear_fwd(x, w)), ("dx", lambda: linear_dx(dy, w)), ("dw", lambda: linear_dw(dy, x))]), flush=True)
