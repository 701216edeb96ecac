"""Graph-timed esgpt::linear_residual_ln (projection + residual + dropout + LayerNorm in one launch) against
esgpt::linear + esgpt::residual_ln at the C2 shapes (out_proj K = 256, c_proj K = 1024; T = 8192, D = 256)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd import ops  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402

esgpt = ops.load()
dev = torch.device("cuda")
t = tickets(dev)
T, D = 8192, 256


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


tag = os.environ.get("ESGPT_GEMM_RESLN_TARGET", "256")
with torch.no_grad():
    for K in (256, 1024):
        x = torch.randn(T, K, device=dev).bfloat16()
        w = (0.05 * torch.randn(D, K, device=dev)).bfloat16()
        bias = torch.randn(D, device=dev)
        r = torch.randn(T, D, device=dev)
        lw, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
        rm = torch.ones(T, dtype=torch.bool, device=dev)
        seed = torch.tensor([7], dtype=torch.int64, device=dev)
        fused = graph_time(lambda: esgpt.linear_residual_ln(x, w, bias, r, lw, lb, rm, 0.1, seed, 1e-5, [], t))
        bare = graph_time(lambda: esgpt.linear_residual_ln(x, w, None, None, lw, lb, None, 0.0, None, 1e-5, [], t))
        print(f"K={K}: fused without bias / residual / mask / dropout {bare:.2f} us", flush=True)
        lin = graph_time(lambda: esgpt.linear(x, w, bias, [], t))
        y = esgpt.linear(x, w, bias, [], t)
        rl = graph_time(lambda: esgpt.residual_ln(r, y, None, lw, lb, rm, 0.1, seed, 1e-5, torch.bfloat16))
        print(f"target={tag} K={K}: fused {fused:.2f} us | linear {lin:.2f} + residual_ln {rl:.2f} = {lin + rl:.2f} us",
              flush=True)
