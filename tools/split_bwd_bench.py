"""Grouped vs split (dW on the weight-gradient stream) projection backwards in a HIP graph: a dependent chain of
c_proj / c_fc backwards (C2 shapes) with a LayerNorm-sized elementwise kernel between them, timed as one replay.
Usage: python tools/split_bwd_bench.py [layers]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from eventstreamgpt_amd import ops
from eventstreamgpt_amd.kernels import join_weight_grads, tickets

esgpt = ops.load()
dev = torch.device("cuda")
T, D, F = 8192, 256, 1024
n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(T, D, device=dev, generator=g).bfloat16()
gact = torch.randn(T, F, device=dev, generator=g).bfloat16()
pre = torch.randn(T, F, device=dev, generator=g).bfloat16()
wfc = (0.05 * torch.randn(F, D, device=dev, generator=g)).bfloat16()
wpj = (0.05 * torch.randn(D, F, device=dev, generator=g)).bfloat16()
dy0 = torch.randn(T, D, device=dev, generator=g).bfloat16()
t0, t1 = tickets(dev), tickets(dev, 1)


def chain(split):
    dy = dy0
    for _ in range(n):
        dz, _, _ = esgpt.linear_bwd(dy, gact, wpj, None, 0, pre, True, True, t0, None, t1 if split else None)
        dx, _, _ = esgpt.linear_bwd(dz, x, wfc, None, -1, None, True, True, t0, None, t1 if split else None)
        dy = (dx.float() * 1.0001).bfloat16()  # a LayerNorm-backward-sized elementwise pass on the main stream
    if split:
        join_weight_grads(dev)
    return dy


res = {}
for split in (False, True, False, True):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain(split)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        out = chain(split)
    gr.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        gr.replay()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    res.setdefault(split, []).append(ms)
    print(f"split={split}: {ms * 1000:.1f} us per chain of {n} (c_proj + c_fc backward + elementwise)", flush=True)
