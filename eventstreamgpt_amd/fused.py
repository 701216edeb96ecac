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
from .kernels import AttentionFn, _timed, next_dropout_seed

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
                                           part.data_ptr(), sums.data_ptr(), L.stream())
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


class WeightShadowFn(torch.autograd.Function):
    """One cat + one cast of the block GEMM weights into a flat compute-dtype buffer, returned as per-layer views
    (Wqkv, Wo, Wfc, Wproj); q, k, v are adjacent so the packed [3D, D] weight is a view. Backward gathers the view
    gradients into one flat f32 buffer (one cat + one cast) and hands each parameter a view of it, instead of
    autograd's per-slice zero-fill + add of the whole flat buffer."""

    @staticmethod
    def forward(ctx, dtype, n_layers: int, *ws):
        flat = torch.cat([w.reshape(-1) for w in ws])
        if dtype != torch.float32:
            flat = flat.to(dtype)
        shapes = [w.shape for w in ws]
        outs, off = [], 0
        for layer in range(n_layers):
            q, k, v, o, fc, pj = shapes[6 * layer: 6 * layer + 6]
            nqkv = q.numel() + k.numel() + v.numel()
            outs.append(flat[off: off + nqkv].view(q[0] + k[0] + v[0], q[1]))
            off += nqkv
            for sh in (o, fc, pj):
                outs.append(flat[off: off + sh.numel()].view(sh))
                off += sh.numel()
        ctx.shapes = shapes
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        ref = next(g for g in gs if g is not None)
        outs_numel = []
        for layer in range(len(ctx.shapes) // 6):
            q, k, v, o, fc, pj = ctx.shapes[6 * layer: 6 * layer + 6]
            outs_numel += [q.numel() + k.numel() + v.numel(), o.numel(), fc.numel(), pj.numel()]
        parts = [g.reshape(-1) if g is not None else torch.zeros(n, dtype=ref.dtype, device=ref.device)
                 for g, n in zip(gs, outs_numel)]
        gflat = torch.cat(parts)
        if gflat.dtype != torch.float32:
            gflat = gflat.float()
        grads, off = [], 0
        for sh in ctx.shapes:
            grads.append(gflat[off: off + sh.numel()].view(sh))
            off += sh.numel()
        return (None, None, *grads)


def weight_shadow(blocks, dtype):
    """Per-layer (Wqkv, Wo, Wfc, Wproj) compute-dtype views of one flat shadow of every block GEMM weight."""
    ws = []
    for b in blocks:
        a = b.attn.attention
        ws += [a.q_proj.weight, a.k_proj.weight, a.v_proj.weight, a.out_proj.weight, b.mlp.c_fc.weight,
               b.mlp.c_proj.weight]
    outs = WeightShadowFn.apply(dtype, len(blocks), *ws)
    return [tuple(outs[4 * i: 4 * i + 4]) for i in range(len(blocks))]


class LinearBiasFn(torch.autograd.Function):
    """z = x @ wᵀ + b in x's dtype (bias in the GEMM epilogue); backward takes the bias gradient with the
    column-sum kernel instead of torch's dim-0 reduction."""

    @staticmethod
    def forward(ctx, x, w, b):
        dt = x.dtype
        wd = w.to(dt)
        z = F.linear(x, wd, b.to(dt))
        ctx.save_for_backward(x, wd)
        ctx.wdtype = w.dtype
        return z

    @staticmethod
    def backward(ctx, dz):
        lib = L.load()
        x, wd = ctx.saved_tensors
        dz = dz.contiguous()
        N, Fo = dz.shape
        dx = dz @ wd if ctx.needs_input_grad[0] else None
        dw = (dz.t() @ x).to(ctx.wdtype) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.needs_input_grad[2]:
            part = torch.empty(lib.esgpt_column_sum_partials(N) * Fo, dtype=torch.float32, device=dz.device)
            db = torch.empty(Fo, dtype=torch.float32, device=dz.device)
            with _timed("column_sum"):
                st = lib.esgpt_column_sum(dz.data_ptr(), L.dtype_code(dz.dtype), N, Fo, part.data_ptr(),
                                          db.data_ptr(), L.stream())
            L.check(st, "column_sum")
        return dx, dw, db


def linear_bias(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``F.linear(x, w, b)`` in the autocast compute dtype with the fused bias-gradient backward (2-D x)."""
    dt = compute_dtype()
    with torch.autocast("cuda", enabled=False):
        return LinearBiasFn.apply(x.to(dt), w, b)


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
    weights = weight_shadow(blocks, dt)
    ln0 = blocks[0].attn.layer_norm
    h, ln = ResidualLNFn.apply(None, input_embeds.reshape(N, D).float().contiguous(), None, ln0.weight, ln0.bias,
                               None, p_in, eps, dt)
    with torch.autocast("cuda", enabled=False):
        for i, blk in enumerate(blocks):
            att = blk.attn.attention
            wqkv, wo, wfc, wpj = weights[i]
            qkv = F.linear(ln, wqkv).view(B, Lq, 3 * D)
            window = att.window_size if att.attention_type == "local" else 0
            o = AttentionFn.apply(qkv, em, em, att.num_heads, window, False, p_att)
            y = F.linear(o.view(N, D), wo)
            h1, ln2 = ResidualLNFn.apply(h, y, att.out_proj.bias, blk.layer_norm.weight, blk.layer_norm.bias, None,
                                         p_res, eps, dt)
            f = F.linear(ln2, wfc)
            g = BiasActFn.apply(f, blk.mlp.c_fc.bias, act)
            y2 = F.linear(g, wpj)
            nxt = blocks[i + 1].attn.layer_norm if i + 1 < len(blocks) else encoder.ln_f
            h, ln = ResidualLNFn.apply(h1, y2, blk.mlp.c_proj.bias, nxt.weight, nxt.bias, rows, p_res, eps, dt)
    return ln.view(B, Lq, D)
