import os, sys, torch
sys.path.insert(0, "/root/repo")
from eventstreamgpt_amd.fused import linear_bwd
T = 8192
for out, inn in [(256, 256), (1024, 256)]:
    x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        linear_bwd(dy, x, w, need_dx=False, need_db=True)
        linear_bwd(dy, x, w, need_db=True)
    torch.cuda.synchronize()
