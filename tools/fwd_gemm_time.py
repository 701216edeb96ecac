"""Graph-timed forward projections of the C2 step (T = 8192 tokens): qkv, out_proj, c_fc (+ bias, GELU, pre
stored), c_proj, the generative head, and c_proj's / out_proj's input-gradient shapes as x·Wtᵀ. Run twice with
ESGPT_GEMM_PANEL=0 / 1 to compare the tile GEMM with the row-panel GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_fwd, linear_fwd_act  # noqa: E402

T = 8192


def graph_time(fn, n=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / n * 1000


tag = "panel" if os.environ.get("ESGPT_GEMM_PANEL", "1") != "0" else "tile"
for name, din, dout, act in [("qkv", 256, 768, -1), ("out_proj", 256, 256, -1), ("c_fc+gelu", 256, 1024, 0),
                             ("c_proj", 1024, 256, -1), ("head", 256, 1624, -1), ("c_proj dX", 256, 1024, -1)]:
    x = torch.randn(T, din, device="cuda").bfloat16()
    w = (0.05 * torch.randn(dout, din, device="cuda")).bfloat16()
    b = torch.randn(dout, device="cuda")
    if act >= 0:
        us = graph_time(lambda: linear_fwd_act(x, w, b, act))
        mb = (T * din * 2 + dout * din * 2 + 2 * T * dout * 2) / 1e6
    else:
        us = graph_time(lambda: linear_fwd(x, w, b))
        mb = (T * din * 2 + dout * din * 2 + T * dout * 2) / 1e6
    tf = 2 * T * din * dout / us / 1e6
    print(f"{tag:5s} {name:10s} {us:7.2f} us  {tf:6.1f} TFLOP/s  {mb / us:5.2f} TB/s ({mb:.1f} MB)", flush=True)
