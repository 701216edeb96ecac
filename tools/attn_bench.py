"""Times the packed-QKV attention kernels (fwd, bwd) at the C2 / C5 layer shapes, with and without dropout, and
prints achieved TFLOP/s against the algorithmic FLOPs (fwd 4*H*hd*T, bwd 8*H*hd*T over allowed (q, k) pairs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.kernels import AttentionFn


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


for (B, L, H, hd) in [(32, 256, 4, 64), (16, 1024, 4, 64), (8, 2048, 8, 128)]:
    D = H * hd
    em = torch.ones(B, L, dtype=torch.bool, device="cuda")
    T = B * L * (L + 1) / 2
    for p in (0.0, 0.1):
        qkv = (0.5 * torch.randn(B, L, 3 * D, device="cuda")).bfloat16().requires_grad_(True)
        o = AttentionFn.apply(qkv, em, em, H, 0, False, p)
        go = torch.randn_like(o)
        tf = t(lambda: AttentionFn.apply(qkv, em, em, H, 0, False, p))
        tb = t(lambda: torch.autograd.grad(AttentionFn.apply(qkv, em, em, H, 0, False, p), qkv, go)) - tf
        print(f"B={B} L={L} H={H} hd={hd} p={p}: fwd {tf:7.1f}us ({4 * H * hd * T / tf / 1e6:6.1f} TF/s)  "
              f"bwd {tb:7.1f}us ({8 * H * hd * T / tb / 1e6:6.1f} TF/s)", flush=True)
