"""Sweeps ESGPT_GEMM_PLAN (wm, wn, splits) for the C2 GEMM shapes; each config in a subprocess."""
import os
import subprocess
import sys

code = r'''
import os, sys, torch
sys.path.insert(0, %r)
from tools.gemm_time import gtime
from eventstreamgpt_amd.fused import linear_dw, linear_dx, linear_fwd
T = 8192
out, inn, op = %d, %d, %r
x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
fn = {"fwd": lambda: linear_fwd(x, w), "dX": lambda: linear_dx(dy, w), "dW": lambda: linear_dw(dy, x)}[op]
print("%%.1f" %% gtime(fn))
'''
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for out, inn in [(768, 256), (256, 256), (1024, 256), (256, 1024)]:
    for op in ("fwd", "dX", "dW"):
        res = []
        plans = ["2,2,1", "2,1,1", "1,1,1"] if op != "dW" else ["1,1,2", "1,1,5", "1,1,10", "2,1,5", "2,1,10", "2,2,5", "2,2,10", "2,2,20"]
        for pl in plans:
            env = dict(os.environ, ESGPT_GEMM_PLAN=pl)
            r = subprocess.run([sys.executable, "-c", code % (repo, out, inn, op)], env=env, capture_output=True, text=True)
            res.append(f"{pl}:{r.stdout.strip() or r.stderr.strip()[-80:]}")
        print((out, inn), op, "  ".join(res), flush=True)
