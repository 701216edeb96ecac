"""Fused CI encoder fast path: residual + dropout + event mask + LayerNorm and bias + activation kernels around
plain (bias-free) GEMMs, with one flat low-precision weight shadow per forward.

Per layer (``InnerBlock``, ``transformer.py:394-461``; encoder loop ``:775-831``):

    qkv = ln @ [Wq;Wk;Wv]ᵀ ; o = attention(qkv) ; y = o @ Woᵀ + b_o
    h1, ln2 = ResidualLN(h, y, dropout, LN2)                               # attn residual
    g = act(ln2 @ Wfcᵀ + b_fc) ; y2 = g @ Wprojᵀ + b_proj
    h, ln = ResidualLN(h1, y2, dropout, event_mask, LN1 of next layer or ln_f)

i.e. 4 GEMMs + attention + 3 fused elementwise kernels per layer, instead of ~20 ATen launches. Parameters are
the modules' own (state_dict unchanged); numerics follow the reference (f32 residual stream and LayerNorm
statistics; GEMM operands in the compute dtype).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib as L

from .kernels import _ops, _timed, attention, batch_args, err_word, next_dropout_seed, terms_list, tickets, tte_lists

_ACTS = {"gelu": 0, "gelu_new": 1, "gelu_pytorch_tanh": 1, "gelu_fast": 1, "relu": 2}


def residual_ln(x, y, bias, ln_w, ln_b, row_mask, p: float, eps: float, out_dtype: torch.dtype, skip_T: int = 0):
    """``esgpt::residual_ln``: h = mask ? x + dropout(y + bias) : 0 ; out = LayerNorm(h). Returns (h f32, out
    out_dtype); differentiable in x, y, bias, ln_w, ln_b (column sums in the backward launch). ``skip_T`` = T: x holds
    T rows per T - 1 output rows and each sequence's first x row is skipped (the static_kv_first residual)."""
    dev = ln_w.device
    seed = next_dropout_seed(dev) if (p > 0 and y is not None) else None
    with _timed("residual_ln_fwd"):
        if skip_T:
            h, out, _mean, _rstd = _ops().residual_ln(x, y, bias, ln_w, ln_b, row_mask, float(p), seed, float(eps),
                                                      out_dtype, int(skip_T))
        else:
            h, out, _mean, _rstd = _ops().residual_ln(x, y, bias, ln_w, ln_b, row_mask, float(p), seed, float(eps),
                                                      out_dtype)
    return h, out


def residual(x, y, row_mask, mask_div: int, skip_T: int, p: float):
    """``esgpt::residual``: h = mask(r) ? x[xr(r)] + dropout(y[r]) : 0 (f32), mask(r) = row_mask[r // mask_div];
    with skip_T = T the rows of x [Bs, T, D] after each first one; x None: a plain dropout of y. Differentiable in x
    and y."""
    seed = next_dropout_seed(y.device) if p > 0 else None
    with _timed("residual_fwd"):
        return _ops().residual(x, y, row_mask, int(mask_div), int(skip_T), float(p), seed)


class ResidualLNFn:
    """Call-compatible name of ``residual_ln``."""

    apply = staticmethod(residual_ln)


def bias_act(f, bias, act: int):
    """``esgpt::bias_act``: g = act(f + bias) for f [N, F] (compute dtype), bias f32 [F]."""
    with _timed("bias_act_fwd"):
        return _ops().bias_act(f, bias, int(act))


class BiasActFn:
    """Call-compatible name of ``bias_act``."""

    apply = staticmethod(bias_act)


def compute_dtype() -> torch.dtype:
    if torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return torch.float32


ENABLED = True  # tests flip this to exercise the module-by-module path
# padded-event row blocks skipped by the dependency-graph projections (esgpt_gemm_row_tiles; exact, tested). Off:
# measured no gain on the C4 step — the mask launches cost ~20-30 us and the skipped ~8 % of the row blocks do not
# shorten the latency-bound launches (profiles/r05_row_tiles_ab.log; bench.py --row-tiles turns it on)
ROW_TILES = False


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
    """``esgpt::gemm_``: out[M, N] (=|+=) alpha·A·B (+ bias) in place (layouts: include/esgpt_amd.h)."""
    with _timed("gemm"):
        _ops().gemm_(out, a_layout, a, lda, b_layout, b, ldb, M, N, K, bias, alpha, bool(accumulate),
                     tickets(a.device))
    return out


def gemm_supported(n_tokens: int, d_in: int, d_out: int) -> bool:
    """Shape constraints of the library GEMMs (esgpt_gemm_bf16 / _f32) for the fwd / dx / dW products of one
    projection: the feature dimensions in 16-B chunks; any token count (the dW product's token dimension is a row
    index of both operands, and edge rows are zero-filled in-kernel)."""
    return d_in % 8 == 0 and d_out % 8 == 0


GEMM_DTYPES = (torch.bfloat16, torch.float32)  # bf16 MFMA, or exact-f32 MFMA (the reference's precision)


def linear_op(x, w_lp, bias, masters, row_tiles=None):
    """``esgpt::linear``: y = x · w_lpᵀ (+ bias) with the bf16 weight shadow ``w_lp``; the backward (one grouped
    launch: dx, f32 dW, db) hands the weight gradient to ``masters`` (the f32 parameters whose row-concatenation
    ``w_lp`` shadows) without a bf16 round trip. ``row_tiles``: the padded-event row-block mask of x's rows
    (``esgpt::row_tiles``): fully padded 64-row blocks skip the forward and dX products."""
    with _timed("gemm"):
        return _ops().linear(x, w_lp, bias, list(masters), tickets(x.device), row_tiles)


def linear_fwd(x, w, bias=None):
    """y[N, out] = x[N, in] · w[out, in]ᵀ (+ bias f32), bf16."""
    return linear_op(x, w, bias, [])


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
    epilogue (``esgpt::linear_act``; the pre-activation is kept for the backward)."""
    with _timed("gemm"):
        return _ops().linear_act(x, w, bias, int(act))


# Launch-shape recorder (bench.py: the in-step roofline of the grouped projection backward over every launch shape)
SHAPES = {"enabled": False, "linear_bwd": []}


def linear_bwd(dy, x, w, alpha=None, act: int = -1, pre=None, need_dx: bool = True, need_db: bool = False):
    """``esgpt::linear_bwd``, one launch for the backward of y = x · wᵀ: dx = alpha·dy·w [· act'(pre)] (bf16),
    dw = alpha·dyᵀ·x (f32) and db = alpha·Σ_rows dy (f32). ``alpha``: optional device scalar.
    Returns (dx | None, dw, db | None)."""
    if SHAPES["enabled"]:
        SHAPES["linear_bwd"].append((dy.shape[0], x.shape[1], dy.shape[1], bool(need_dx), int(act), bool(need_db)))
    with _timed("gemm"):
        dx, dw, db = _ops().linear_bwd(dy, x, w, alpha, int(act), pre, bool(need_dx), bool(need_db), tickets(x.device))
    return (dx if need_dx else None), dw, (db if need_db else None)


def column_sum(x):
    """``esgpt::column_sum``: f32 column sums of x [N, F] (fixed order)."""
    with _timed("column_sum"):
        return _ops().column_sum(x)


class ProjFn:
    """Call-compatible name of ``linear_op``: ``ProjFn.apply(x, w_lp, bias, *params)``."""

    @staticmethod
    def apply(x, w_lp, bias, *params):
        return linear_op(x, w_lp, bias, params)


def proj(x, w_lp, bias, params, row_tiles=None):
    """Projection through the HIP GEMM (bf16 shadow, or the f32 weights themselves in the reference-precision mode)
    when the shapes allow it, else ``F.linear`` on the (differentiable) compute-dtype weights."""
    if w_lp is not None and w_lp.dtype in GEMM_DTYPES and gemm_supported(x.shape[0], x.shape[1], w_lp.shape[0]):
        return linear_op(x.to(w_lp.dtype).contiguous(), w_lp, bias, params, row_tiles)
    w = params[0] if len(params) == 1 else torch.cat(list(params), 0)
    dt = x.dtype
    return F.linear(x, w.to(dt), None if bias is None else bias.to(dt))


def mlp_op(x, w_fc, w_pj, b_fc, act: int, p_fc, p_pj, b_pj=None, row_tiles=None):
    """``esgpt::mlp``: InnerMLP (transformer.py:378-391): y = act(x · W_fcᵀ + b_fc) · W_projᵀ (+ b_proj) in two
    GEMM launches (c_fc's bias + activation in its epilogue, the bf16 pre-activation kept; c_proj's bias in its
    epilogue) and two grouped backward launches (c_proj: d(pre) = (dy · W_proj) · act'(pre) in the dX epilogue, +
    dW_proj + db_proj; c_fc: dx + dW_fc + db_fc, the bias gradients as row sums inside the dW products). The residual
    dropout belongs to the following residual_ln. ``w_fc`` / ``w_pj`` are the bf16 shadows; the f32 parameters
    ``p_fc`` / ``p_pj`` receive the gradients."""
    with _timed("gemm"):
        y, _pre, _g = _ops().mlp(x, w_fc, w_pj, b_fc, b_pj, int(act), p_fc, p_pj, tickets(x.device), row_tiles)
    return y


class MLPFn:
    """Call-compatible name of ``mlp_op``."""

    apply = staticmethod(mlp_op)


def mlp(x, w_fc, w_pj, fc, pj, act: int, with_bias: bool = False, row_tiles=None):
    """InnerMLP (c_proj's bias included only with ``with_bias``): ``mlp_op`` when the bf16 GEMM shapes allow it,
    else proj + bias_act + proj."""
    if (w_fc is not None and w_fc.dtype in GEMM_DTYPES
            and gemm_supported(x.shape[0], x.shape[1], w_fc.shape[0])):
        return mlp_op(x.to(w_fc.dtype).contiguous(), w_fc, w_pj, fc.bias, act, fc.weight, pj.weight,
                      pj.bias if with_bias else None, row_tiles)
    f = proj(x, w_fc, None, (fc.weight,))
    g = bias_act(f, fc.bias, act)
    return proj(g, w_pj, pj.bias if with_bias else None, (pj.weight,))


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
    if dtype in GEMM_DTYPES:  # one esgpt::pack launch (a cat + a cast otherwise)
        code = L.BF16 if dtype == torch.bfloat16 else L.F32
        flat = _ops().pack([w.detach().contiguous() for w in ws], [len(ws)], [0], [code])[0]
    else:
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
        if dt in GEMM_DTYPES and x.is_cuda:
            with torch.no_grad():  # one esgpt::pack launch: the row-concatenated weights in the compute dtype
                code = L.BF16 if dt == torch.bfloat16 else L.F32
                w_lp = _ops().pack([p.detach().float().contiguous() for p in params], [len(params)], [0], [code])[0]
                w_lp = w_lp.view(-1, params[0].shape[1])
            return proj(x.to(dt), w_lp, b, params)
        return proj(x.to(dt), None, b, params)


def head_loss_op(xc, xt, batch, terms, tte, shift: int, n_levels: int, cw, cb, tw, tb):
    """``esgpt::head_loss``: bf16 generative heads + fused losses in one autograd node (model_output.py:1253-1721):
    z = x · W_padᵀ + b_pad with the HIP GEMM (the head's output columns padded to a multiple of 8 with zero
    weights), the loss kernel computes the losses AND d(loss)/dz, and the backward scales every gradient by the
    incoming d(total) straight from device memory (the GEMM's alpha pointer) — no logits-sized scaling pass, no host
    sync. ``xt`` / ``tw`` / ``tb`` are None / empty when the TTE columns are part of the content head (CI). Returns
    f32 [n_terms + 2] like ``output_loss``."""
    wcode = L.BF16 if xc.dtype == torch.bfloat16 else L.F32  # the logits' (and GEMM operands') dtype
    with torch.no_grad():
        # every padded head weight / bias copy in one esgpt::pack launch: [W_c | 0] (compute dtype), [b_c | 0] f32
        # and in the logits' dtype (the position-0 logits when shifted), [W_t | 0], [b_t | 0] f32
        D = cw[0].shape[1]
        nc = sum(w.shape[0] for w in cw)
        pc = (-nc) % 8
        srcs = [w.detach() for w in cw] + [b.detach() for b in cb] + ([b.detach() for b in cb] if shift else [])
        groups, tails, codes = [len(cw), len(cb)], [pc * D, pc], [wcode, L.F32]
        if shift:
            groups.append(len(cb))
            tails.append(pc)
            codes.append(wcode)
        if tw:
            nt = sum(w.shape[0] for w in tw)
            pt = (-nt) % 8
            srcs += [w.detach() for w in tw] + [b.detach() for b in tb]
            groups += [len(tw), len(tb)]
            tails += [pt * D, pt]
            codes += [wcode, L.F32]
        out = _ops().pack([t.float().contiguous() for t in srcs], groups, tails, codes)
        wc, bc = out[0].view(nc + pc, D), out[1]
        zb = out[2] if shift else None
        wt = out[-2].view(-1, D) if tw else None
        bt = out[-1] if tw else None
    ti, tf = tte_lists(tte)
    dev = xc.device
    with _timed("output_loss"):
        losses, _, _, _ = _ops().head_loss(xc, xt, *batch_args(batch), terms_list(terms), ti, tf, int(shift),
                                           int(n_levels), wc, bc, wt, bt, list(cw), list(cb), list(tw), list(tb),
                                           err_word(dev), tickets(dev), zb)
    return losses


def head_losses(xc, xt, batch, terms, tte, shift, n_levels, cmods, tmods):
    """Generative heads + losses through ``esgpt::head_loss`` (bf16 compute, or exact f32 in the reference-precision
    mode) — None if the shapes do not fit the HIP GEMM (the caller then uses the module-by-module path)."""
    D = xc.shape[1]
    dt = compute_dtype()
    if dt not in GEMM_DTYPES or D % 8 or not xc.is_cuda:
        return None
    cw = [m.weight for m in cmods]
    cb = [m.bias for m in cmods]
    tw = [m.weight for m in tmods]
    tb = [m.bias for m in tmods]
    xc = xc.to(dt).contiguous()
    xt = None if xt is None else xt.to(dt).contiguous()
    with torch.autocast("cuda", enabled=False):
        return head_loss_op(xc, xt, batch, terms, tte, shift, n_levels, cw, cb, tw, tb)


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
    weights = weight_shadow(blocks, dt) if dt in GEMM_DTYPES else [(None,) * 4] * len(blocks)
    ln0 = blocks[0].attn.layer_norm
    h, ln = residual_ln(None, input_embeds.reshape(N, D).float().contiguous(), None, ln0.weight, ln0.bias,
                        None, p_in, eps, dt)
    with torch.autocast("cuda", enabled=False):
        for i, blk in enumerate(blocks):
            att = blk.attn.attention
            wqkv, wo, wfc, wpj = weights[i]
            qkv = proj(ln, wqkv, None, (att.q_proj.weight, att.k_proj.weight, att.v_proj.weight)).view(B, Lq, 3 * D)
            window = att.window_size if att.attention_type == "local" else 0
            o = attention(qkv, em, em, att.num_heads, window, False, p_att)
            # the projections' biases in the GEMM epilogues (as the reference's bf16 nn.Linear), their gradients as
            # row sums inside the backward dW products
            y = proj(o.view(N, D), wo, att.out_proj.bias, (att.out_proj.weight,))
            h1, ln2 = residual_ln(h, y, None, blk.layer_norm.weight, blk.layer_norm.bias, None, p_res, eps, dt)
            y2 = mlp(ln2, wfc, wpj, blk.mlp.c_fc, blk.mlp.c_proj, act, with_bias=True)
            nxt = blocks[i + 1].attn.layer_norm if i + 1 < len(blocks) else encoder.ln_f
            h, ln = residual_ln(h1, y2, None, nxt.weight, nxt.bias, rows, p_res, eps, dt)
    return ln.view(B, Lq, D)


def block_fused_supported(blk, hidden: torch.Tensor) -> bool:
    """An ``InnerBlock`` can run through the HIP kernels (bf16 autocast or f32 on a HIP tensor, GEMM-friendly
    feature widths; any token count)."""
    if not (hidden.is_cuda and compute_dtype() in GEMM_DTYPES and ENABLED):
        return False
    cfg_act = getattr(blk.mlp, "act_name", None)
    D = hidden.shape[-1]
    F_ = blk.mlp.c_fc.out_features
    return cfg_act in _ACTS and D % 8 == 0 and F_ % 8 == 0 and D <= 1024 and blk.attn.attention.head_dim <= 128


def inner_block_fused(blk, hidden: torch.Tensor, key_padding_mask, static_kv_first: bool, out_row_mask=None,
                      out_mask_div: int = 1) -> torch.Tensor:
    """``InnerBlock.forward`` (``transformer.py:409-461``, pre-LN attention + MLP with residuals) through the HIP
    kernels: LayerNorm, one packed-QKV GEMM, attention, out_proj with its bias + residual dropout + the second
    LayerNorm fused, the MLP GEMMs (bias + activation epilogue), the last residual + dropout as one kernel — the same
    pieces as the fused CI encoder, for a stand-alone block (the NA sequence and dependency-graph modules).
    ``hidden`` [Bs, T, D] f32; returns [Bs, T - skf, D] f32. ``out_row_mask`` (bool, one entry per ``out_mask_div``
    output rows): rows of masked-out events are zeros (StructuredAttention's event-mask wheres, fused)."""
    att = blk.attn.attention
    Bs, T, D = hidden.shape
    skf = 1 if static_kv_first else 0
    eps = float(blk.layer_norm.eps)
    train = blk.training
    p_res = float(att.resid_dropout.p) if train else 0.0
    p_att = att.attn_dropout_p if train else 0.0
    dt = compute_dtype()  # bf16, or f32 (the reference precision: exact-f32 MFMA GEMMs)
    wqkv, wo, wfc, wpj = weight_shadow([blk], dt)[0]
    ln1 = blk.attn.layer_norm
    x2 = hidden.reshape(Bs * T, D).float().contiguous()
    kpm = None if key_padding_mask is None else key_padding_mask.contiguous()
    qpm = None if (kpm is None or static_kv_first) else kpm
    window = att.window_size if att.attention_type == "local" else 0
    Tq = T - skf
    # Rows of masked-out events (the padded events of the dependency graph, which the reference compacts away,
    # structured_attention.py:162-165): their outputs are zeroed and their gradients are zero, so the projections
    # skip the 64-row blocks holding nothing else (forward and dX products; esgpt_gemm_row_tiles). Row-wise valid
    # results are bitwise unchanged.
    tiles_in = tiles_out = None
    if (ROW_TILES and out_row_mask is not None and hidden.is_cuda and out_mask_div == Tq
            and out_row_mask.numel() * Tq == Bs * Tq):
        em = out_row_mask.reshape(-1)
        tiles_in, tiles_out = _ops().row_tiles(em, T), _ops().row_tiles(em, Tq)
    with torch.autocast("cuda", enabled=False):
        # h0 (= x2) feeds the block's residual: its gradient comes back into this LayerNorm's backward as dh_in
        # (one kernel), not as a second gradient of x2 that autograd would add
        h0, ln = residual_ln(None, x2, None, ln1.weight, ln1.bias, None, 0.0, eps, dt)
        qkv = proj(ln, wqkv, None, (att.q_proj.weight, att.k_proj.weight, att.v_proj.weight),
                   tiles_in).view(Bs, T, 3 * D)
        o = attention(qkv, kpm, qpm, att.num_heads, window, static_kv_first, p_att)
        y = proj(o.reshape(Bs * Tq, D), wo, att.out_proj.bias, (att.out_proj.weight,), tiles_out)
        # the residual rows: every row of h0, or (static_kv_first) all but each sequence's first, mapped in-kernel
        h1, ln2 = residual_ln(h0, y, None, blk.layer_norm.weight, blk.layer_norm.bias, None, p_res, eps, dt,
                              skip_T=T if skf else 0)
        y2 = mlp(ln2, wfc, wpj, blk.mlp.c_fc, blk.mlp.c_proj, _ACTS[blk.mlp.act_name], with_bias=True,
                 row_tiles=tiles_out)
        out = residual(h1, y2, out_row_mask, out_mask_div, 0, p_res)
    return out.view(Bs, Tq, D)
