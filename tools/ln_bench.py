"""Residual + LayerNorm kernels at the C2 step's shape (N = B*L = 8192 rows, D = 256, bf16 branch / output, f32
residual stream, dropout 0.1): graph-replayed launch time and algorithmic HBM bytes.

    ESGPT_LN_BWD_ROWS=4 python tools/ln_bench.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import graph_time_ms  # noqa: E402
from eventstreamgpt_amd import _lib as L  # noqa: E402
from eventstreamgpt_amd.kernels import tickets  # noqa: E402


def main():
    lib = L.load()
    dev = torch.device("cuda")
    N, D = 8192, 256
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, D, device=dev, generator=g)
    y = torch.randn(N, D, device=dev, generator=g).bfloat16()
    bias = torch.randn(D, device=dev, generator=g)
    w = torch.rand(D, device=dev, generator=g) + 0.5
    b = torch.randn(D, device=dev, generator=g)
    seed = torch.tensor([7], dtype=torch.int64, device=dev)
    h = torch.empty(N, D, device=dev)
    out = torch.empty(N, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(N, device=dev)
    rstd = torch.empty(N, device=dev)
    dout = torch.randn(N, D, device=dev, generator=g).bfloat16()
    dh = torch.randn(N, D, device=dev, generator=g)
    dx = torch.empty(N, D, device=dev)
    dy = torch.empty(N, D, device=dev, dtype=torch.bfloat16)
    part = torch.empty(lib.esgpt_residual_ln_partials(N) * 3 * D, device=dev)
    sums = torch.empty(3 * D, device=dev)
    cnt = tickets(dev)
    assert lib.esgpt_residual_ln_counters(N) <= cnt.numel()

    def fwd():
        L.check(lib.esgpt_residual_ln_fwd(x.data_ptr(), y.data_ptr(), L.BF16, bias.data_ptr(), None, 0.1,
                                          seed.data_ptr(), w.data_ptr(), b.data_ptr(), 1e-5, N, D, h.data_ptr(),
                                          out.data_ptr(), L.BF16, mean.data_ptr(), rstd.data_ptr(), L.stream()),
                "ln_fwd")

    def bwd():
        L.check(lib.esgpt_residual_ln_bwd(dh.data_ptr(), dout.data_ptr(), L.BF16, h.data_ptr(), mean.data_ptr(),
                                          rstd.data_ptr(), w.data_ptr(), None, 0.1, seed.data_ptr(), N, D,
                                          dx.data_ptr(), dy.data_ptr(), L.BF16, part.data_ptr(), sums.data_ptr(),
                                          cnt.data_ptr(), L.stream()), "ln_bwd")

    fwd()
    torch.cuda.synchronize()
    tf = graph_time_ms(fwd)
    tb = graph_time_ms(bwd)
    fwd_bytes = N * D * (4 + 2 + 4 + 2)  # x, y in; h, out
    bwd_bytes = N * D * (4 + 2 + 4 + 4 + 2)  # dh, dout, h in; dx, dy out
    print(json.dumps({"rows_per_wave": os.environ.get("ESGPT_LN_BWD_ROWS", "4"),
                      "fwd_us": round(tf * 1e3, 2), "fwd_GBs": round(fwd_bytes / tf / 1e6, 1),
                      "bwd_us": round(tb * 1e3, 2), "bwd_GBs": round(bwd_bytes / tb / 1e6, 1)}))


if __name__ == "__main__":
    main()
