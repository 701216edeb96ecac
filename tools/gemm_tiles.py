"""Projection GEMMs at the C2 step's shapes (T = 8192) under one tile configuration (the ESGPT_GEMM_TILE_FWD / _DX /
_DW tuning hooks of csrc/gemm.hip, read once per process): forward (c_fc with its GELU epilogue, the rest plain)
and the grouped backward pair, graph-replayed; one JSON line per shape plus the step-weighted total (6 layers of
qkv / out / c_fc / c_proj + the head), and a numerics check of every product against torch f32.

    ESGPT_GEMM_TILE_FWD=22 python tools/gemm_tiles.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_bwd, linear_fwd, linear_fwd_act  # noqa: E402
from tools.gemm_time import gtime  # noqa: E402

# (out, in, layers per step, GELU epilogue on the forward / its gradient on the backward)
SHAPES = [(768, 256, 6, False), (256, 256, 6, False), (1024, 256, 6, True), (256, 1024, 6, True),
          (1624, 256, 1, False)]


def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))


def main():
    T = 8192
    cfg = {k: os.environ.get("ESGPT_GEMM_TILE_" + k, "11") for k in ("FWD", "DX", "DW")}
    g = torch.Generator(device="cuda").manual_seed(0)
    tot_f = tot_b = 0.0
    worst = 0.0
    for out, inn, n, act in SHAPES:
        x = torch.randn(T, inn, device="cuda", generator=g).bfloat16()
        w = (torch.randn(out, inn, device="cuda", generator=g) * inn ** -0.5).bfloat16()
        b = torch.randn(out, device="cuda", generator=g)
        dy = torch.randn(T, out, device="cuda", generator=g).bfloat16()
        # GELU: c_fc's forward epilogue (out = 1024), c_proj's dX epilogue (in = 1024)
        if act and out > inn:
            fwd = lambda: linear_fwd_act(x, w, b, 0)  # noqa: E731
        else:
            fwd = lambda: linear_fwd(x, w, b)  # noqa: E731
        pre = torch.randn(T, inn, device="cuda", generator=g).bfloat16() if act and inn > out else None
        tf = gtime(fwd)
        tb = gtime(lambda: linear_bwd(dy, x, w, act=0 if pre is not None else -1, pre=pre, need_db=True))
        # numerics vs torch f32 (plain products: dX = dY W, dW = dYᵀ X, db = Σ dY)
        y = linear_fwd(x, w, b)
        ref_y = x.float() @ w.float().t() + b
        dx, dw, db = linear_bwd(dy, x, w, need_db=True)
        worst = max(worst, rel(y, ref_y), rel(dx, dy.float() @ w.float()), rel(dw, dy.float().t() @ x.float()),
                    rel(db, dy.float().sum(0)))
        fl = 2.0 * T * out * inn
        tot_f += n * tf
        tot_b += n * tb
        print(json.dumps({"cfg": cfg, "out": out, "in": inn, "fwd_us": round(tf, 2),
                          "fwd_tflops": round(fl / tf / 1e6, 1), "bwd_us": round(tb, 2),
                          "bwd_tflops": round(2 * fl / tb / 1e6, 1)}), flush=True)
    print(json.dumps({"cfg": cfg, "step_fwd_us": round(tot_f, 1), "step_bwd_us": round(tot_b, 1),
                      "max_rel_err": worst}), flush=True)


if __name__ == "__main__":
    main()
