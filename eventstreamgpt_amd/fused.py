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
    return ENABLED and cfg.activation_function in _ACTS and cfg.hidden_size <= 1024


def weight_shadow(blocks, dtype):
    """One cat (+ one cast) of every block GEMM weight; returns per-layer views (Wqkv, Wo, Wfc, Wproj)."""
    ws, shapes = [], []
    for b in blocks:
        a = b.attn.attention
        for w in (a.q_proj.weight, a.k_proj.weight, a.v_proj.weight, a.out_proj.weight, b.mlp.c_fc.weight,
                  b.mlp.c_proj.weight):
            ws.append(w.reshape(-1))
            shapes.append(w.shape)
    flat = torch.cat(ws)
    if dtype != torch.float32:
        flat = flat.to(dtype)
    out, off, i = [], 0, 0
    for _ in blocks:
        start = off
        views = []
        for _k in range(6):
            n = shapes[i].numel()
            views.append(flat[off: off + n].view(shapes[i]))
            off += n
            i += 1
        wq = views[0]
        # q, k, v are adjacent in the flat buffer: the packed [3D, D] weight is a view, no extra copy.
        wqkv = flat[start: start + 3 * wq.numel()].view(3 * wq.shape[0], wq.shape[1])
        out.append((wqkv, views[3], views[4], views[5]))
    return out


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
