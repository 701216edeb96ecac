"""GPU time of the HIP projection GEMM at the C2 step's shapes: 20 launches captured in a HIP graph, replayed
(no host launch overhead in the number). Prints us per call and achieved TFLOP/s / GB/s (algorithmic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_dw, linear_dx, linear_fwd  # noqa: E402


def gtime(fn, n=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
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
    return a.elapsed_time(b) * 1e3 / (n * reps)


def main():
    T = 8192
    tot = 0.0
    for out, inn in [(768, 256), (256, 256), (1024, 256), (256, 1024), (1624, 256)]:
        x = torch.randn(T, inn, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(out, inn, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, out, device="cuda", dtype=torch.bfloat16)
        fl = 2 * T * out * inn
        res = []
        for name, fn, byts in [("fwd", lambda: linear_fwd(x, w), 2 * (T * inn + out * inn + T * out)),
                               ("dX", lambda: linear_dx(dy, w), 2 * (T * out + out * inn + T * inn)),
                               ("dW", lambda: linear_dw(dy, x), 2 * (T * out + T * inn) + 4 * out * inn)]:
            us = gtime(fn)
            if out != 1624:
                tot += us
            res.append(f"{name} {us:6.1f}us ({fl / us / 1e6:5.0f} TF/s, {byts / us / 1e3:5.0f} GB/s)")
        print((out, inn), "  ".join(res), flush=True)
    print(f"sum over one layer's 12 projection GEMMs: {tot:.1f} us", flush=True)


if __name__ == "__main__":
    main()
