"""Streamed-tile GEMM (gemm_stream_kernel) check + timing on the C2 projection shapes, under the tools build
(ESGPT_GEMM_STREAM selects the configuration, read once per process): forward y = x·Wᵀ + b (+ GELU with pre), and
the input-gradient form dx = dy·W (· act'(pre)). Errors vs a torch f32 reference of the same bf16 operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402

T = int(os.environ.get("T", "8192"))
lib = L.load()
tag = os.environ.get("ESGPT_GEMM_STREAM", "off")


def graph_time(fn, n=20, reps=10):
    fn()
    torch.cuda.synchronize()
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


def gelu(z):
    return torch.nn.functional.gelu(z)


torch.manual_seed(0)
worst = 0.0
for name, din, dout, act in [("qkv", 256, 768, -1), ("out_proj", 256, 256, -1), ("c_fc+gelu", 256, 1024, 0),
                             ("c_proj", 1024, 256, -1), ("head", 256, 1624, -1), ("odd", 264, 200, -1)]:
    Tn = T if name != "odd" else T - 77
    x = torch.randn(Tn, din, device="cuda").bfloat16()
    w = (0.05 * torch.randn(dout, din, device="cuda")).bfloat16()
    b = torch.randn(dout, device="cuda")
    y = torch.empty(Tn, dout, device="cuda", dtype=torch.bfloat16)
    pre = torch.empty_like(y) if act >= 0 else None

    def fwd():
        L.check(lib.esgpt_linear_fwd(x.data_ptr(), din, w.data_ptr(), Tn, din, dout, b.data_ptr(), act, L.ptr(pre),
                                     y.data_ptr(), dout, L.stream()), "fwd")

    us = graph_time(fwd)
    fwd()
    ref = x.float() @ w.float().t() + b
    err = ((pre if act >= 0 else y).float() - ref).abs().max().item() / ref.abs().max().item()
    if act >= 0:
        e2 = (y.float() - gelu(pre.float())).abs().max().item()
        err = max(err, e2 / 10)
    worst = max(worst, err)
    tf = 2 * Tn * din * dout / us / 1e6
    print(f"{tag:5s} fwd {name:10s} {us:7.2f} us {tf:6.1f} TF  err {err:.2e}", flush=True)
print(f"{tag} worst rel err {worst:.2e}", flush=True)
assert worst < 2e-2
