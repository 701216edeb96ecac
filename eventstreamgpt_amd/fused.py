"""Fused CI encoder fast path: residual + dropout + event mask + LayerNorm and bias + activation kernels around
plain (bias-free) GEMMs, with one flat low-precision weight shadow per forward.

Per layer (``InnerBlock``, ``transformer.py:394-461``; encoder loop ``:775-831``):

    qkv = ln @ [Wq;Wk;Wv]ᵀ ; o = attention(qkv) ; y = o @ Woᵀ
    h1, ln2 = ResidualLN(h, y + b_o, dropout, LN2)                         # attn residual
    g = act(ln2 @ Wfcᵀ + b_fc) ; y2 = g @ Wprojᵀ
    h, ln = ResidualLN(h1, y2 + b_proj, dropout, event_mask, LN1 of next layer or ln_f)

i.e. 4 GEMMs + attention + 3 fused elementwise kernels per layer, instead of ~20 ATen launches. Parameters are
the modules' own (state_dict unchanged); numerics follow the reference (f32 residual stream and LayerNorm
statistics; GEMM operands in the compute dtype).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib as L
import ctypes

from .kernels import AttentionFn, _timed, err_word, next_dropout_seed, tickets

_ACTS = {"gelu": 0, "gelu_new": 1, "gelu_pytorch_tanh": 1, "gelu_fast": 1, "relu": 2}


class ResidualLNFn(torch.autograd.Function):
    """h = mask ? x + dropout(y + bias) : 0 ; out = LayerNorm(h). Returns (h f32, out out_dtype)."""

    @staticmethod
    def forward(ctx, x, y, bias, ln_w, ln_b, row_mask, p: float, eps: float, out_dtype: torch.dtype):
        lib = L.load()
        ref = x if x is not None else y
        N, D = ref.shape
        dev = ref.device
        h = torch.empty(N, D, dtype=torch.float32, device=dev)
        out = torch.empty(N, D, dtype=out_dtype, device=dev)
        mean = torch.empty(N, dtype=torch.float32, device=dev)
        rstd = torch.empty(N, dtype=torch.float32, device=dev)
        seed = next_dropout_seed(dev) if (p > 0 and y is not None) else None
        y_dtype = y.dtype if y is not None else torch.float32
        with _timed("residual_ln_fwd"):
            st = lib.esgpt_residual_ln_fwd(L.ptr(x), L.ptr(y), L.dtype_code(y_dtype), L.ptr(bias), L.ptr(row_mask),
                                           float(p), L.ptr(seed), ln_w.data_ptr(), ln_b.data_ptr(), float(eps), N, D,
                                           h.data_ptr(), out.data_ptr(), L.dtype_code(out_dtype), mean.data_ptr(),
                                           rstd.data_ptr(), L.stream())
        L.check(st, "residual_ln_fwd")
        ctx.save_for_backward(h, mean, rstd, ln_w, row_mask, seed)
        ctx.set_materialize_grads(False)
        ctx.meta = (x is not None, y is not None, bias is not None, y_dtype, out_dtype, float(p))
        return h, out

    @staticmethod
    def backward(ctx, dh, dout):
        lib = L.load()
        h, mean, rstd, ln_w, row_mask, seed = ctx.saved_tensors
        has_x, has_y, has_bias, y_dtype, out_dtype, p = ctx.meta
        N, D = h.shape
        dev = h.device
        if dout is None:
            dout = torch.zeros(N, D, dtype=out_dtype, device=dev)
        dout = dout.contiguous().to(out_dtype)
        dh_in = None if dh is None else dh.contiguous().float()
        dx = torch.empty(N, D, dtype=torch.float32, device=dev) if has_x else None
        dy = torch.empty(N, D, dtype=y_dtype, device=dev) if has_y else None
        nb = lib.esgpt_residual_ln_partials(N)
        part = torch.empty(nb * 3 * D, dtype=torch.float32, device=dev)
        sums = torch.empty(3, D, dtype=torch.float32, device=dev)
        with _timed("residual_ln_bwd"):
            st = lib.esgpt_residual_ln_bwd(L.ptr(dh_in), dout.data_ptr(), L.dtype_code(out_dtype), h.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), ln_w.data_ptr(), L.ptr(row_mask),
                                           p, L.ptr(seed), N, D, L.ptr(dx), L.ptr(dy), L.dtype_code(y_dtype),
                                           part.data_ptr(), sums.data_ptr(), tickets(dev).data_ptr(), L.stream())
        L.check(st, "residual_ln_bwd")
        return dx, dy, (sums[2] if has_bias else None), sums[0], sums[1], None, None, None, None


class BiasActFn(torch.autograd.Function):
    """g = act(f + bias) for f [N, F] (compute dtype), bias f32 [F]."""

    @staticmethod
    def forward(ctx, f, bias, act: int):
        lib = L.load()
        f = f.contiguous()
        N, Fd = f.shape
        g = torch.empty_like(f)
        with _timed("bias_act_fwd"):
            st = lib.esgpt_bias_act_fwd(f.data_ptr(), bias.data_ptr(), act, N, Fd, g.data_ptr(),
                                        L.dtype_code(f.dtype), L.stream())
        L.check(st, "bias_act_fwd")
        ctx.save_for_backward(f, bias)
        ctx.act = act
        return g

    @staticmethod
    def backward(ctx, dg):
        lib = L.load()
        f, bias = ctx.saved_tensors
        N, Fd = f.shape
        dg = dg.contiguous().to(f.dtype)
        dz = torch.empty_like(f)
        part = torch.empty(lib.esgpt_bias_act_partials(N) * Fd, dtype=torch.float32, device=f.device)
        dbias = torch.empty(Fd, dtype=torch.float32, device=f.device)
        with _timed("bias_act_bwd"):
            st = lib.esgpt_bias_act_bwd(dg.data_ptr(), f.data_ptr(), bias.data_ptr(), ctx.act, N, Fd, dz.data_ptr(),
                                        part.data_ptr(), dbias.data_ptr(), L.dtype_code(f.dtype), L.stream())
        L.check(st, "bias_act_bwd")
        return dz, dbias, None


def compute_dtype() -> torch.dtype:
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return torch.float32


ENABLED = True  # tests flip this to exercise the module-by-module path


def fused_supported(encoder) -> bool:
    cfg = encoder.config
    return (ENABLED and cfg.activation_function in _ACTS and cfg.hidden_size <= 1024 and cfg.hidden_size % 4 == 0
            and cfg.intermediate_size % 4 == 0)


# ----------------------------------------------------------------------------------------------------------------
# Projection GEMMs (csrc/gemm.hip): y = x·Wᵀ (+ b) [+ act], and one grouped launch per projection backward
# (dx = dy·W [· act'], dW = dyᵀ·x and db = Σ dy written straight to f32)
# ----------------------------------------------------------------------------------------------------------------
def _gemm(a, a_layout: int, lda: int, b, b_layout: int, ldb: int, M: int, N: int, K: int, out, bias=None,
          accumulate: bool = False, alpha=None):
    lib = L.load()
    nbytes = lib.esgpt_gemm_workspace(M, N, K)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=a.device) if nbytes else None
    cnt = tickets(a.device)
    if nbytes and lib.esgpt_gemm_counters(M, N) > cnt.numel():
        raise RuntimeError("eventstreamgpt_amd: GEMM tile grid exceeds the ticket array")
    with _timed("gemm"):
        st = lib.esgpt_gemm_bf16(a_layout, a.data_ptr(), lda, b_layout, b.data_ptr(), ldb, M, N, K, L.ptr(bias),
                                 L.ptr(alpha), out.data_ptr(), out.stride(0), L.dtype_code(out.dtype),
                                 int(accumulate), L.ptr(ws), nbytes, cnt.data_ptr(), L.stream())
    L.check(st, "gemm")
    return out


def gemm_supported(n_tokens: int, d_in: int, d_out: int) -> bool:
    """Shape constraints of esgpt_gemm_bf16 for the fwd / dx / dW products of one projection."""
    return n_tokens % 8 == 0 and d_in % 8 == 0 and d_out % 8 == 0


def linear_fwd(x, w, bias=None):
    """y[N, out] = x[N, in] · w[out, in]ᵀ (+ bias f32), bf16."""
    N, din = x.shape
    y = torch.empty(N, w.shape[0], dtype=x.dtype, device=x.device)
    return _gemm(x, L.GEMM_K_CONTIG, din, w, L.GEMM_K_CONTIG, din, N, w.shape[0], din, y, bias)


def linear_dx(dy, w):
    """dx[N, in] = dy[N, out] · w[out, in], bf16."""
    N, dout = dy.shape
    dx = torch.empty(N, w.shape[1], dtype=dy.dtype, device=dy.device)
    return _gemm(dy, L.GEMM_K_CONTIG, dout, w, L.GEMM_MN_CONTIG, w.shape[1], N, w.shape[1], dout, dx)


def linear_dw(dy, x):
    """dW[out, in] = dy[N, out]ᵀ · x[N, in] in f32 (the parameters' dtype; no bf16 rounding of the gradient)."""
    N, dout = dy.shape
    din = x.shape[1]
    dw = torch.empty(dout, din, dtype=torch.float32, device=dy.device)
    return _gemm(dy, L.GEMM_MN_CONTIG, dout, x, L.GEMM_MN_CONTIG, din, dout, din, N, dw)


def linear_fwd_act(x, w, bias, act: int):
    """(pre, y): pre = x · wᵀ + bias (bf16) and y = act(pre) — c_fc with its bias and activation in the GEMM
    epilogue (the pre-activation is kept for the backward)."""
    lib = L.load()
    T, din = x.shape
    dout = w.shape[0]
    pre = torch.empty(T, dout, dtype=x.dtype, device=x.device)
    y = torch.empty_like(pre)
    with _timed("gemm"):
        st = lib.esgpt_linear_fwd(x.data_ptr(), x.stride(0), w.data_ptr(), T, din, dout, L.ptr(bias), int(act),
                                  pre.data_ptr(), y.data_ptr(), y.stride(0), L.stream())
    L.check(st, "linear_fwd")
    return pre, y


# Launch-shape recorder (bench.py: the in-step roofline of the grouped projection backward over every launch shape)
SHAPES = {"enabled": False, "linear_bwd": []}


def linear_bwd(dy, x, w, alpha=None, act: int = -1, pre=None, need_dx: bool = True, need_db: bool = False):
    """One launch for the backward of y = x · wᵀ: dx = alpha·dy·w [· act'(pre)] (bf16), dw = alpha·dyᵀ·x (f32) and
    db = alpha·Σ_rows dy (f32). ``alpha``: optional device scalar. Returns (dx | None, dw, db | None)."""
    lib = L.load()
    T, dout = dy.shape
    din = x.shape[1]
    if SHAPES["enabled"]:
        SHAPES["linear_bwd"].append((T, din, dout, bool(need_dx), int(act), bool(need_db)))
    dev = dy.device
    dw = torch.empty(dout, din, dtype=torch.float32, device=dev)
    dx = torch.empty(T, din, dtype=dy.dtype, device=dev) if need_dx else None
    db = torch.empty(dout, dtype=torch.float32, device=dev) if need_db else None
    nbytes = lib.esgpt_linear_bwd_workspace(T, din, dout, int(need_dx))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev) if nbytes else None
    cnt = tickets(dev)
    if nbytes and lib.esgpt_gemm_counters(dout, din) > cnt.numel():
        raise RuntimeError("eventstreamgpt_amd: GEMM tile grid exceeds the ticket array")
    with _timed("gemm"):
        st = lib.esgpt_linear_bwd(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(), T, din, dout,
                                  L.ptr(alpha), int(act), L.ptr(pre), 0 if pre is None else pre.stride(0), L.ptr(dx),
                                  0 if dx is None else dx.stride(0), dw.data_ptr(), L.ptr(db), L.ptr(ws), nbytes,
                                  cnt.data_ptr(), L.stream())
    L.check(st, "linear_bwd")
    return dx, dw, db


def column_sum(x):
    lib = L.load()
    N, Fo = x.shape
    part = torch.empty(lib.esgpt_column_sum_partials(N) * Fo, dtype=torch.float32, device=x.device)
    out = torch.empty(Fo, dtype=torch.float32, device=x.device)
    with _timed("column_sum"):
        st = lib.esgpt_column_sum(x.data_ptr(), L.dtype_code(x.dtype), N, Fo, part.data_ptr(), out.data_ptr(),
                                  L.stream())
    L.check(st, "column_sum")
    return out


class ProjFn(torch.autograd.Function):
    """y = x · w_lpᵀ (+ bias) where ``w_lp`` is a no-grad bf16 shadow of the row-concatenation of ``params`` (f32).
    Backward: one grouped launch for dx = dy · w_lp, dW = dyᵀ · x (directly in f32, handed to each parameter as a
    row slice) and dbias (a row sum inside the dW product). No bf16 gradient round trip, no cast kernels."""

    @staticmethod
    def forward(ctx, x, w_lp, bias, *params):
        x = x.contiguous()
        y = linear_fwd(x, w_lp, bias)
        ctx.save_for_backward(x, w_lp)
        ctx.rows = [p.shape[0] for p in params]
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        dx, dw, db = linear_bwd(dy.contiguous(), x, w, need_dx=ctx.needs_input_grad[0], need_db=need_db)
        grads = list(torch.split(dw, ctx.rows, 0))
        return (dx, None, db, *grads)


def proj(x, w_lp, bias, params):
    """Projection through the HIP GEMM when the shapes allow it, else ``F.linear`` on the (differentiable)
    compute-dtype weights."""
    if w_lp is not None and w_lp.dtype == torch.bfloat16 and gemm_supported(x.shape[0], x.shape[1], w_lp.shape[0]):
        return ProjFn.apply(x.to(torch.bfloat16), w_lp, bias, *params)
    w = params[0] if len(params) == 1 else torch.cat(list(params), 0)
    dt = x.dtype
    return F.linear(x, w.to(dt), None if bias is None else bias.to(dt))


class MLPFn(torch.autograd.Function):
    """InnerMLP (transformer.py:378-391) up to c_proj's bias: y = act(x · W_fcᵀ + b_fc) · W_projᵀ in two GEMM
    launches (c_fc's bias + activation in its epilogue; the bf16 pre-activation is kept) and two grouped backward
    launches (c_proj: d(pre) = (dy · W_proj) · act'(pre) in the dX epilogue, + dW_proj; c_fc: dx + dW_fc + db_fc as a
    row sum inside its dW product). c_proj's bias and the residual dropout belong to the following ResidualLNFn.
    ``w_fc`` / ``w_pj`` are the bf16 shadows; the f32 parameters ``p_fc`` / ``p_pj`` receive the gradients."""

    @staticmethod
    def forward(ctx, x, w_fc, w_pj, b_fc, act: int, p_fc, p_pj):
        x = x.contiguous()
        pre, g = linear_fwd_act(x, w_fc, b_fc, act)
        y = linear_fwd(g, w_pj)
        ctx.save_for_backward(x, w_fc, w_pj, pre, g)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_fc, w_pj, pre, g = ctx.saved_tensors
        dz, dw_pj, _ = linear_bwd(dy.contiguous(), g, w_pj, act=ctx.act, pre=pre)
        dx, dw_fc, db_fc = linear_bwd(dz, x, w_fc, need_dx=ctx.needs_input_grad[0], need_db=True)
        return dx, None, None, db_fc, None, dw_fc, dw_pj


def mlp(x, w_fc, w_pj, fc, pj, act: int):
    """InnerMLP without c_proj's bias: ``MLPFn`` when the bf16 GEMM shapes allow it, else proj + BiasActFn + proj."""
    if (w_fc is not None and w_fc.dtype == torch.bfloat16
            and gemm_supported(x.shape[0], x.shape[1], w_fc.shape[0])):
        return MLPFn.apply(x.to(torch.bfloat16), w_fc, w_pj, fc.bias, act, fc.weight, pj.weight)
    f = proj(x, w_fc, None, (fc.weight,))
    g = BiasActFn.apply(f, fc.bias, act)
    return proj(g, w_pj, None, (pj.weight,))


@torch.no_grad()
def weight_shadow(blocks, dtype):
    """One cat + one cast of every block GEMM weight into a flat compute-dtype buffer (no autograd: the gradients
    come from ProjFn straight into the f32 parameters). Returns per-layer (Wqkv, Wo, Wfc, Wproj) views; q, k, v
    are adjacent, so the packed [3D, D] weight is a view."""
    ws = []
    for b in blocks:
        a = b.attn.attention
        ws += [a.q_proj.weight, a.k_proj.weight, a.v_proj.weight, a.out_proj.weight, b.mlp.c_fc.weight,
               b.mlp.c_proj.weight]
    flat = torch.cat([w.reshape(-1) for w in ws]).to(dtype)
    out, off = [], 0
    for i in range(len(blocks)):
        q, k, v, o, fc, pj = ws[6 * i: 6 * i + 6]
        nqkv = q.numel() + k.numel() + v.numel()
        views = [flat[off: off + nqkv].view(q.shape[0] + k.shape[0] + v.shape[0], q.shape[1])]
        off += nqkv
        for w in (o, fc, pj):
            views.append(flat[off: off + w.numel()].view(w.shape))
            off += w.numel()
        out.append(tuple(views))
    return out


def linear_bias(x: torch.Tensor, params, biases) -> torch.Tensor:
    """Head projection: x · [params]ᵀ + [biases] in the autocast compute dtype (2-D x). ``params`` / ``biases``
    are lists of the modules' weights and biases, row-concatenated."""
    dt = compute_dtype()
    b = torch.cat(list(biases), 0) if len(biases) > 1 else biases[0]
    with torch.autocast("cuda", enabled=False):
        if dt == torch.bfloat16:
            with torch.no_grad():
                w_lp = torch.cat([p.detach() for p in params], 0).to(dt)
            return proj(x.to(dt), w_lp, b, params)
        return proj(x.to(dt), None, b, params)


_ZPAD: dict = {}


def _pad_rows(ts, mult: int = 8):
    """Row-concatenation of ``ts`` (same dtype / trailing dim) padded with zero rows to a multiple of ``mult``
    (one cat kernel; the zero block is cached)."""
    n = sum(t.shape[0] for t in ts)
    pad = (-n) % mult
    if pad:
        t0 = ts[0]
        key = (pad, tuple(t0.shape[1:]), t0.dtype, t0.device)
        z = _ZPAD.get(key)
        if z is None:
            z = torch.zeros((pad,) + tuple(t0.shape[1:]), dtype=t0.dtype, device=t0.device)
            _ZPAD[key] = z
        ts = list(ts) + [z]
    return torch.cat(list(ts), 0) if len(ts) > 1 else ts[0]


class HeadLossFn(torch.autograd.Function):
    """bf16 generative heads + fused losses in one autograd node (model_output.py:1253-1721 through
    ``OutputLossFn``'s kernel): z = x · W_padᵀ + b_pad with the HIP GEMM (the head's output columns padded to a
    multiple of 8 with zero weights), the loss kernel computes the losses AND d(loss)/dz, and the backward scales
    every gradient by the incoming d(total) straight from device memory (the GEMM's alpha pointer) — no logits-
    sized scaling pass, no host sync. ``xt`` / TTE params are None when the TTE columns are part of the content
    head (CI). Returns f32 [n_terms + 2] like ``OutputLossFn``."""

    @staticmethod
    def forward(ctx, xc, xt, bv, terms, tte, shift: int, n_levels: int, n_cw: int, n_tw: int, *wb):
        lib = L.load()
        cw, cb = wb[:n_cw], wb[n_cw: 2 * n_cw]
        tw, tb = wb[2 * n_cw: 2 * n_cw + n_tw], wb[2 * n_cw + n_tw:]
        with torch.no_grad():
            wc = _pad_rows([w.detach() for w in cw]).to(torch.bfloat16)
            bc = _pad_rows([b.detach().float() for b in cb]).contiguous()
            zc = linear_fwd(xc, wc, bc)
            if n_tw:
                wt = _pad_rows([w.detach() for w in tw]).to(torch.bfloat16)
                bt = _pad_rows([b.detach().float() for b in tb]).contiguous()
                zt = linear_fwd(xt, wt, bt)
            else:
                wt = bt = zt = None
        zc_bias = bc.to(torch.bfloat16) if shift else None
        n_terms = len(terms)
        arr = (L.EsgptLossTerm * max(1, n_terms))(*terms)
        zt_ = zc if zt is None else zt
        dzc = torch.empty_like(zc)
        dzt = dzc if zt is None else torch.empty_like(zt)
        dbias = torch.empty(bv.B, zc.shape[1], dtype=torch.float32, device=zc.device) if shift else None
        losses = torch.empty(n_terms + 2, dtype=torch.float32, device=zc.device)
        nbytes = lib.esgpt_output_loss_workspace(bv.B, bv.L, n_terms)
        ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=zc.device)
        with _timed("output_loss"):
            st = lib.esgpt_output_loss(bv.ref, zc.data_ptr(), zc.shape[1], n_levels, shift, L.ptr(zc_bias),
                                       zt_.data_ptr(), zt_.shape[1], L.BF16, arr, n_terms, ctypes.byref(tte),
                                       dzc.data_ptr(), dzt.data_ptr(), L.ptr(dbias), losses.data_ptr(), ws.data_ptr(),
                                       nbytes, err_word(zc.device).data_ptr(), L.stream())
        L.check(st, "output_loss")
        ctx.save_for_backward(xc, xt, wc, wt, dzc, None if zt is None else dzt, dbias)
        ctx.rows = ([w.shape[0] for w in cw], [w.shape[0] for w in tw])
        ctx.n = (n_cw, n_tw)
        return losses

    @staticmethod
    def backward(ctx, g):
        xc, xt, wc, wt, dzc, dzt, dbias = ctx.saved_tensors
        n_cw, n_tw = ctx.n
        rows_c, rows_t = ctx.rows
        g = g.contiguous()
        alpha = g[-1:]  # d(total): read by the GEMMs from device memory
        dxc, dwc, dbc = linear_bwd(dzc, xc, wc, alpha=alpha, need_db=True)
        if dbias is not None:
            dbc = dbc + dbias.sum(0) * alpha
        n_real_c = sum(rows_c)
        gw_c = list(torch.split(dwc[:n_real_c], rows_c, 0))
        gb_c = list(torch.split(dbc[:n_real_c], rows_c, 0))
        dxt, gw_t, gb_t = None, [], []
        if n_tw:
            dxt, dwt, dbt = linear_bwd(dzt, xt, wt, alpha=alpha, need_db=True)
            n_real_t = sum(rows_t)
            gw_t = list(torch.split(dwt[:n_real_t], rows_t, 0))
            gb_t = list(torch.split(dbt[:n_real_t], rows_t, 0))
        return (dxc, dxt, None, None, None, None, None, None, None, *gw_c, *gb_c, *gw_t, *gb_t)


def head_losses(xc, xt, bv, terms, tte, shift, n_levels, cmods, tmods):
    """Generative heads + losses through ``HeadLossFn`` (bf16 compute) — None if the shapes do not fit the HIP
    GEMM (the caller then uses the module-by-module path)."""
    D = xc.shape[1]
    if compute_dtype() != torch.bfloat16 or D % 8 or xc.shape[0] % 8 or (xt is not None and xt.shape[0] % 8):
        return None
    cw = [m.weight for m in cmods]
    cb = [m.bias for m in cmods]
    tw = [m.weight for m in tmods]
    tb = [m.bias for m in tmods]
    xc = xc.to(torch.bfloat16).contiguous()
    xt = None if xt is None else xt.to(torch.bfloat16).contiguous()
    with torch.autocast("cuda", enabled=False):
        return HeadLossFn.apply(xc, xt, bv, terms, tte, shift, n_levels, len(cw), len(tw), *cw, *cb, *tw, *tb)


def ci_encoder_fused(encoder, batch, input_embeds: torch.Tensor, input_dropout: float):
    """Runs the CI encoder's blocks + ln_f through the fused path. ``input_embeds`` is the masked input embedding
    BEFORE input dropout. Returns ln_f(hidden) [B, L, D] in the compute dtype."""
    cfg = encoder.config
    dt = compute_dtype()
    B, Lq, D = input_embeds.shape
    N = B * Lq
    em = batch.event_mask
    rows = em.reshape(N).contiguous()
    train = encoder.training
    p_in = float(input_dropout) if train else 0.0
    p_res = float(cfg.resid_dropout) if train else 0.0
    p_att = float(cfg.attention_dropout) if train else 0.0
    eps = float(cfg.layer_norm_epsilon)
    act = _ACTS[cfg.activation_function]
    blocks = list(encoder.h)
    weights = weight_shadow(blocks, dt) if dt == torch.bfloat16 else [(None,) * 4] * len(blocks)
    ln0 = blocks[0].attn.layer_norm
    h, ln = ResidualLNFn.apply(None, input_embeds.reshape(N, D).float().contiguous(), None, ln0.weight, ln0.bias,
                               None, p_in, eps, dt)
    with torch.autocast("cuda", enabled=False):
        for i, blk in enumerate(blocks):
            att = blk.attn.attention
            wqkv, wo, wfc, wpj = weights[i]
            qkv = proj(ln, wqkv, None, (att.q_proj.weight, att.k_proj.weight, att.v_proj.weight)).view(B, Lq, 3 * D)
            window = att.window_size if att.attention_type == "local" else 0
            o = AttentionFn.apply(qkv, em, em, att.num_heads, window, False, p_att)
            y = proj(o.view(N, D), wo, None, (att.out_proj.weight,))
            h1, ln2 = ResidualLNFn.apply(h, y, att.out_proj.bias, blk.layer_norm.weight, blk.layer_norm.bias, None,
                                         p_res, eps, dt)
            y2 = mlp(ln2, wfc, wpj, blk.mlp.c_fc, blk.mlp.c_proj, act)
            nxt = blocks[i + 1].attn.layer_norm if i + 1 < len(blocks) else encoder.ln_f
            h, ln = ResidualLNFn.apply(h1, y2, blk.mlp.c_proj.bias, nxt.weight, nxt.bias, rows, p_res, eps, dt)
    return ln.view(B, Lq, D)


def block_fused_supported(blk, hidden: torch.Tensor) -> bool:
    """An ``InnerBlock`` can run through the HIP kernels (bf16 autocast on a HIP tensor, GEMM-friendly shapes)."""
    if not (hidden.is_cuda and compute_dtype() == torch.bfloat16 and ENABLED):
        return False
    cfg_act = getattr(blk.mlp, "act_name", None)
    D = hidden.shape[-1]
    F_ = blk.mlp.c_fc.out_features
    n_tok = hidden.numel() // D
    return (cfg_act in _ACTS and D % 8 == 0 and F_ % 8 == 0 and n_tok % 8 == 0 and D <= 1024
            and blk.attn.attention.head_dim <= 128)


def inner_block_fused(blk, hidden: torch.Tensor, key_padding_mask, static_kv_first: bool) -> torch.Tensor:
    """``InnerBlock.forward`` (``transformer.py:409-461``, pre-LN attention + MLP with residuals) through the HIP
    kernels: LayerNorm, one packed-QKV GEMM, attention, out_proj with its bias + residual dropout + the second
    LayerNorm fused, the MLP GEMMs (bias + activation epilogue) — the same pieces as the fused CI encoder, for a
    stand-alone block (the NA sequence and dependency-graph modules). ``hidden`` [Bs, T, D] f32; returns
    [Bs, T - skf, D] f32."""
    att = blk.attn.attention
    Bs, T, D = hidden.shape
    skf = 1 if static_kv_first else 0
    eps = float(blk.layer_norm.eps)
    train = blk.training
    p_res = float(att.resid_dropout.p) if train else 0.0
    p_att = att.attn_dropout_p if train else 0.0
    dt = torch.bfloat16
    wqkv, wo, wfc, wpj = weight_shadow([blk], dt)[0]
    ln1 = blk.attn.layer_norm
    x2 = hidden.reshape(Bs * T, D).float().contiguous()
    kpm = None if key_padding_mask is None else key_padding_mask.contiguous()
    qpm = None if (kpm is None or static_kv_first) else kpm
    window = att.window_size if att.attention_type == "local" else 0
    with torch.autocast("cuda", enabled=False):
        _, ln = ResidualLNFn.apply(None, x2, None, ln1.weight, ln1.bias, None, 0.0, eps, dt)
        qkv = proj(ln, wqkv, None, (att.q_proj.weight, att.k_proj.weight, att.v_proj.weight)).view(Bs, T, 3 * D)
        o = AttentionFn.apply(qkv, kpm, qpm, att.num_heads, window, static_kv_first, p_att)
        Tq = T - skf
        y = proj(o.reshape(Bs * Tq, D), wo, None, (att.out_proj.weight,))
        res = hidden[:, skf:, :].reshape(Bs * Tq, D).float().contiguous()
        h1, ln2 = ResidualLNFn.apply(res, y, att.out_proj.bias, blk.layer_norm.weight, blk.layer_norm.bias, None,
                                     p_res, eps, dt)
        y2 = mlp(ln2, wfc, wpj, blk.mlp.c_fc, blk.mlp.c_proj, _ACTS[blk.mlp.act_name])
        out = h1 + F.dropout(y2.float() + blk.mlp.c_proj.bias, p=p_res, training=train)
    return out.view(Bs, Tq, D)
