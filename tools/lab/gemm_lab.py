"""Times the LDS-DMA GEMM lab variants (tools/lab/gemm_lab.hip) against the product forward projection on the C2
forward shapes (T = 8192), graph-replayed, and checks each against torch. Tools only."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from eventstreamgpt_amd.fused import linear_fwd  # noqa: E402

lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libgemmlab.so"))
lab.lab_fwd.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
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
    best = 1e9
    for _ in range(3):
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps / n * 1000)
    return best


variants = [int(v) for v in sys.argv[1:]] or list(range(12))
for name, din, dout in [("qkv", 256, 768), ("out_proj", 256, 256), ("c_fc", 256, 1024), ("c_proj", 1024, 256),
                        ("head1664", 256, 1664)]:
    x = torch.randn(T, din, device="cuda").bfloat16()
    w = (0.05 * torch.randn(dout, din, device="cuda")).bfloat16()
    b = torch.randn(dout, device="cuda")
    ref = (x.float() @ w.float().t() + b)
    fl = 2 * T * din * dout
    us = graph_time(lambda: linear_fwd(x, w, b))
    print(f"{name:9s} prod      {us:7.2f} us {fl / us / 1e6:6.0f} TF", flush=True)
    for v in variants:
        y = torch.empty(T, dout, device="cuda", dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream
        rc = lab.lab_fwd(v, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), T, dout, din, st)
        if rc != 0:
            print(f"{name:9s} v{v:<2d} skipped ({rc})")
            continue
        torch.cuda.synchronize()
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        us = graph_time(lambda: lab.lab_fwd(v, x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), T, dout, din,
                                             torch.cuda.current_stream().cuda_stream))
        print(f"{name:9s} v{v:<2d}      {us:7.2f} us {fl / us / 1e6:6.0f} TF  err {err:.1e}", flush=True)
