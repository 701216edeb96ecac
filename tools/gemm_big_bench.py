"""Graph-timed projections of a C3 layer (T = 16,384 tokens, d = 512, F = 2,048): the forward products (qkv,
out_proj, c_fc + GELU with the pre-activation stored, c_proj) and each one's grouped backward (dX [· GELU'] + dW
+ db). Run under the tools build with ESGPT_GEMM_BIG = 0 (tile GEMM) / 128 / 256 / unset (the product rule):

    bash tools/with_tuning.sh env ESGPT_GEMM_BIG=0 python tools/gemm_big_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eventstreamgpt_amd.fused import linear_bwd, linear_dx, linear_fwd, linear_fwd_act  # noqa: E402

PEAK = 2500.0
T = int(os.environ.get("T", "16384"))
D, F = int(os.environ.get("D", "512")), int(os.environ.get("F", "2048"))


def graph_time(fn, n=10, reps=10):
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


tag = os.environ.get("ESGPT_GEMM_BIG", "rule")
tot_f = tot_b = fl_f = fl_b = 0.0
for name, din, dout, act in [("qkv", D, 3 * D, -1), ("out_proj", D, D, -1), ("c_fc", D, F, 0), ("c_proj", F, D, -1)]:
    g = torch.Generator(device="cuda").manual_seed(din + dout)
    x = torch.randn(T, din, device="cuda", generator=g).bfloat16()
    w = (0.05 * torch.randn(dout, din, device="cuda", generator=g)).bfloat16()
    b = torch.randn(dout, device="cuda", generator=g)
    dy = torch.randn(T, dout, device="cuda", generator=g).bfloat16()
    pre = torch.randn(T, din, device="cuda", generator=g).bfloat16()
    alpha = torch.ones(1, device="cuda")
    if act >= 0:
        uf = graph_time(lambda: linear_fwd_act(x, w, b, act))
    else:
        uf = graph_time(lambda: linear_fwd(x, w, b))
    # backward of this Linear; c_proj's dX carries c_fc's GELU' (act on its input side)
    bact = 0 if name == "c_proj" else -1
    ub = graph_time(lambda: linear_bwd(dy, x, w, alpha=alpha, act=bact, pre=pre if bact >= 0 else None,
                                       need_dx=True, need_db=True))
    ux = graph_time(lambda: linear_dx(dy, w))  # dX alone (no activation gradient)
    uw = graph_time(lambda: linear_bwd(dy, x, w, alpha=alpha, need_dx=False, need_db=True))  # dW + db alone
    ff, fb = 2.0 * T * din * dout, 4.0 * T * din * dout
    tot_f += uf
    tot_b += ub
    fl_f += ff
    fl_b += fb
    print(f"{tag:5s} {name:9s} fwd {uf:8.2f} us {ff / uf / 1e6:7.1f} TF/s ({ff / uf / 1e6 / PEAK:.3f})   "
          f"bwd {ub:8.2f} us {fb / ub / 1e6:7.1f} TF/s ({fb / ub / 1e6 / PEAK:.3f})   "
          f"dX {ux:7.2f} us ({ff / ux / 1e6 / PEAK:.3f})  dW {uw:7.2f} us ({ff / uw / 1e6 / PEAK:.3f})", flush=True)
print(f"{tag:5s} layer     fwd {tot_f:8.2f} us ({fl_f / tot_f / 1e6 / PEAK:.3f})   bwd {tot_b:8.2f} us "
      f"({fl_b / tot_b / 1e6 / PEAK:.3f})", flush=True)
if os.environ.get("SQUARE", "1") == "1":  # the guide's reference shape: 8192^3 bf16 (random operands)
    S = 8192
    x = torch.rand(S, S, device="cuda").mul_(2).sub_(1).bfloat16()
    w = torch.rand(S, S, device="cuda").mul_(2).sub_(1).bfloat16()
    try:
        us = graph_time(lambda: linear_fwd(x, w), n=3, reps=5)
    except RuntimeError as e:  # the tile GEMM does not take K = 8192 unsplit
        print(f"{tag:5s} square    fwd: {e}")
        sys.exit(0)
    print(f"{tag:5s} square    fwd {us:8.2f} us {2.0 * S ** 3 / us / 1e6:7.1f} TF/s ({2.0 * S ** 3 / us / 1e6 / PEAK:.3f})",
          flush=True)
