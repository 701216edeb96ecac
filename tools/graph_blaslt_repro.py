"""Round-1 NA graph-replay divergence, isolated: PyTorch-ROCm Linear layers (bf16 autocast, with bias) captured into a
HIP graph the way TrainStep captured the round-1 NA blocks (two warm-up passes on a side stream, then
torch.cuda.graph), replayed over fresh inputs with host allocations between replays, against eager gradients.

Variants (one line of JSON each):
  blas      hipblaslt (PyTorch-ROCm default for these GEMMs) | rocblas (torch.backends.cuda.preferred_blas_library)
  churn     allocate / fill / free device memory on the host between replays (what TrainStep's callers did)
The bias gradient of Linear backward is the reduction the round-1 diagnostics found corrupted (c_proj.bias / c_fc.bias).

    python tools/graph_blaslt_repro.py
"""
import json

import torch
import torch.nn as nn


ACT = {"name": "gelu"}


def make(seed=0):
    torch.manual_seed(seed)
    act = {"gelu": nn.GELU(), "none": nn.Identity(), "relu": nn.ReLU()}[ACT["name"]]
    return nn.Sequential(nn.Linear(256, 1024), act, nn.Linear(1024, 256)).cuda()


def grads_of(m):
    return [p.grad.detach().float().clone() for p in m.parameters()]


AUTOCAST = {"on": True}


def fwd_bwd(m, x):
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False, enabled=AUTOCAST["on"]):
        y = m(x)
    loss = y.float().square().mean()
    loss.backward()
    return loss.detach()


def run(blas: str, churn: bool, steps: int = 6, autocast: bool = True, x_grad: bool = False, act: str = "gelu"):
    torch.backends.cuda.preferred_blas_library(blas)
    ACT["name"] = act
    AUTOCAST["on"] = autocast
    xs = [torch.randn(8192, 256, device="cuda", generator=torch.Generator("cuda").manual_seed(100 + i))
          .requires_grad_(x_grad) for i in range(steps)]
    m = make()
    want, want_loss = [], []
    for x in xs:
        for p in m.parameters():
            p.grad = None
        want_loss.append(float(fwd_bwd(m, x)))
        want.append(grads_of(m))
    m = make()
    static = xs[0].detach().clone().requires_grad_(x_grad)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in m.parameters():
                p.grad = None
            fwd_bwd(m, static)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for p in m.parameters():
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sloss = fwd_bwd(m, static)
    worst, lerr, stale = [], [], []
    for i, x in enumerate(xs):
        with torch.no_grad():
            static.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        got = grads_of(m)
        worst.append([float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, want[i])])
        stale.append([float((a - b).abs().max() / (b.abs().max() + 1e-30)) for a, b in zip(got, want[0])])
        lerr.append(abs(float(sloss) - want_loss[i]) / abs(want_loss[i]))
        if churn:  # host-side allocations and frees between replays
            junk = [torch.full((1 << 22,), 1e38, device="cuda") for _ in range(8)]
            junk += [torch.empty(1 << 20, device="cuda").uniform_() for _ in range(8)]
            del junk
    # a race between captured nodes (a reader not ordered after its producer) reads the previous replay's leftovers:
    # replaying the same input twice would then be exact the second time
    twice = []
    for _ in range(2):
        with torch.no_grad():
            static.copy_(xs[1])
        g.replay()
        torch.cuda.synchronize()
        twice.append([f"{float((a - b).abs().max() / (b.abs().max() + 1e-30)):.1e}" for a, b in zip(grads_of(m), want[1])])
    names = [n for n, _ in m.named_parameters()]
    return {"same_input_replayed_twice": twice, "act": ACT["name"],"blas": blas, "churn": churn, "autocast": autocast, "x_requires_grad": x_grad, "loss_rel_err": [f"{e:.1e}" for e in lerr],
            "grad_rel_err_per_param": {n: [f"{w[j]:.1e}" for w in worst] for j, n in enumerate(names)},
            "vs_capture_input_grads": {n: [f"{w[j]:.1e}" for w in stale] for j, n in enumerate(names)}}


def column_sum_case(rows: int, cols: int, steps: int = 4, dtype=torch.float32):
    """The bias-gradient reduction alone: y = x.sum(0) captured, replayed over fresh x."""
    xs = [torch.randn(rows, cols, device="cuda", generator=torch.Generator("cuda").manual_seed(7 + i)).to(dtype)
          for i in range(steps)]
    static = xs[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            static.sum(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = static.sum(0)
    errs = []
    for x in xs:
        static.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        want = x.sum(0)
        errs.append(float((y.float() - want.float()).abs().max() / want.float().abs().max()))
    return {"case": f"x[{rows},{cols}] {dtype}.sum(0) replayed", "rel_err_per_replay": [f"{e:.1e}" for e in errs]}


def gelu_bias_case(steps: int = 4, x_grad: bool = False):
    """One Linear + GELU (f32, no autocast), loss = mean(y^2): which gradient goes wrong under replay, and whether
    it equals the capture input's gradient (a stale, not re-executed node)."""
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 1024).cuda()
    xs = [torch.randn(8192, 256, device="cuda", generator=torch.Generator("cuda").manual_seed(50 + i))
          for i in range(steps)]

    def fb(x):
        y = torch.nn.functional.gelu(lin(x))
        loss = y.square().mean()
        loss.backward()

    want = []
    for x in xs:
        lin.weight.grad = lin.bias.grad = None
        fb(x.requires_grad_(x_grad))
        want.append((lin.weight.grad.clone(), lin.bias.grad.clone()))
    static = xs[0].detach().clone().requires_grad_(x_grad)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            lin.weight.grad = lin.bias.grad = None
            fb(static)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    lin.weight.grad = lin.bias.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb(static)
    out = []
    for i, x in enumerate(xs):
        with torch.no_grad():
            static.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        r = lambda a, b: f"{float((a - b).abs().max() / b.abs().max()):.1e}"
        out.append({"dW": r(lin.weight.grad, want[i][0]), "db": r(lin.bias.grad, want[i][1]),
                    "db_vs_capture_input": r(lin.bias.grad, want[0][1]),
                    "db_accumulated": r(lin.bias.grad, sum(w[1] for w in want[: i + 1]))})
    return {"case": f"Linear+GELU f32, x.requires_grad={x_grad}", "per_replay": out}


def memset_sweep_case(replays: int = 4):
    """memset_node_case over sizes and byte offsets, plus the same buffer zeroed by a fill kernel (zero_())."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    out = {}
    for nbytes in (64, 1024, 16384, 1 << 20):
        for off in (0, 4, 256):
            for how in ("memset", "fill"):
                base = torch.zeros((off + nbytes) // 4 + 64, device="cuda")
                buf = base[off // 4: off // 4 + nbytes // 4]
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    if how == "memset":
                        st = torch.cuda.current_stream().cuda_stream
                        hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(nbytes),
                                           ctypes.c_void_p(st))
                    else:
                        buf.zero_()
                    buf.add_(1.0)
                vals = []
                for _ in range(replays):
                    g.replay()
                    torch.cuda.synchronize()
                    vals.append(float(buf.max()))
                out[f"{how} {nbytes}B @+{off}"] = vals
    return {"case": "memset / fill node + add 1, max after each replay (1.0 = node re-ran)", "results": out}


def linear_db_by_gemm_case(steps: int = 4):
    """The failing Linear -> GELU -> Linear case with every bias gradient computed as a GEMM (dYᵀ·1) instead of
    ATen's cross-block column-sum reduction (whose semaphores hipMemsetAsync zeroes)."""

    class Lin(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            return x @ w.t() + b

        @staticmethod
        def backward(ctx, g):
            x, w = ctx.saved_tensors
            ones = torch.ones(g.shape[0], 1, device=g.device, dtype=g.dtype)
            return g @ w, g.t() @ x, (g.t() @ ones).squeeze(1)

    torch.manual_seed(0)
    l0, l2 = nn.Linear(256, 1024).cuda(), nn.Linear(1024, 256).cuda()
    ps = [l0.weight, l0.bias, l2.weight, l2.bias]
    xs = [torch.randn(8192, 256, device="cuda", generator=torch.Generator("cuda").manual_seed(100 + i))
          for i in range(steps)]

    def fb(x):
        h = torch.nn.functional.gelu(Lin.apply(x, l0.weight, l0.bias))
        Lin.apply(h, l2.weight, l2.bias).square().mean().backward()

    want = []
    for x in xs:
        for p in ps:
            p.grad = None
        fb(x)
        want.append([p.grad.clone() for p in ps])
    static = xs[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for p in ps:
                p.grad = None
            fb(static)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for p in ps:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb(static)
    errs = []
    for i, x in enumerate(xs):
        static.copy_(x)
        g.replay()
        torch.cuda.synchronize()
        errs.append([f"{float((p.grad - w).abs().max() / w.abs().max()):.1e}" for p, w in zip(ps, want[i])])
    return {"case": "Linear->GELU->Linear, bias gradients as GEMMs (no ATen reduction)", "per_replay_[w0,b0,w2,b2]": errs}


def memset_node_case(replays: int = 3):
    """hipMemsetAsync captured into a graph, followed by a kernel adding 1: after each replay the buffer holds 1 if
    the memset node re-runs, the replay count if it does not."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    buf = torch.zeros(1 << 16, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream().cuda_stream
        rc = hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, ctypes.c_size_t(buf.numel() * 4),
                                ctypes.c_void_p(st))
        buf.add_(1.0)
    vals = []
    for _ in range(replays):
        g.replay()
        torch.cuda.synchronize()
        vals.append(float(buf.max()))
    return {"case": "hipMemsetAsync node + add 1, replayed", "rc": rc, "buffer_after_each_replay": vals}


if __name__ == "__main__":
    for case in (lambda: column_sum_case(8192, 1024), lambda: column_sum_case(8192, 256),
                 lambda: column_sum_case(8192, 1024, dtype=torch.bfloat16), memset_node_case, memset_sweep_case,
                 linear_db_by_gemm_case,
                 lambda: gelu_bias_case(x_grad=False), lambda: gelu_bias_case(x_grad=True)):
        try:
            print(json.dumps(case()), flush=True)
        except Exception as e:
            print(json.dumps({"error": repr(e)[:300]}), flush=True)
    for blas, churn, ac, xg, act in (("hipblaslt", False, True, False, "gelu"), ("hipblaslt", False, False, False, "gelu"),
                                     ("cublas", False, False, False, "gelu"), ("hipblaslt", True, True, False, "gelu"),
                                     ("hipblaslt", False, False, False, "none"), ("hipblaslt", False, False, False, "relu")):
        if True:
            try:
                print(json.dumps(run(blas, churn, autocast=ac, x_grad=xg, act=act)), flush=True)
            except Exception as e:  # report and continue with the next variant
                print(json.dumps({"blas": blas, "churn": churn, "error": repr(e)[:300]}), flush=True)
