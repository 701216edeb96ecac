"""Forward projection GEMM time vs K (and vs plain copy roofline) at M = 8192 tokens: how much of a launch is the
K loop and how much is fixed (prologue latency, epilogue stores, launch)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_fwd  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402


def main():
    T = 8192
    for N in (256, 1024):
        for K in (64, 128, 256, 512, 1024):
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            us = gtime(lambda: linear_fwd(x, w))
            byt = 2 * (T * K + N * K + T * N)
            print(f"N={N:5d} K={K:5d}: {us:6.2f} us  {2 * T * N * K / us / 1e6:6.1f} TF  {byt / us / 1e3:6.0f} GB/s",
                  flush=True)
        y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
        src = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        us = gtime(lambda: y.copy_(src))
        print(f"copy [{T},{N}] bf16: {us:6.2f} us {4 * T * N / us / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
