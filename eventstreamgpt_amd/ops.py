"""``torch.ops.esgpt``: the PyTorch-ROCm custom operators of this package.

The operators are defined and implemented in C++ (``csrc/torch_ops.cpp`` → ``libesgpt_torch.so``:
``TORCH_LIBRARY(esgpt, m)`` with HIP implementations that call the C ABI of ``libesgpt_amd.so``). This module loads
that library and registers, per operator, a fake (meta) kernel — output shapes / dtypes without running anything,
for fake tensors, ``torch.compile`` and export — and, for the differentiable ones, the autograd formula
(``torch.library.register_autograd``) whose backward calls the matching ``*_bwd`` operator.

Differentiable operators and the reference code they replace:

====================  =====================================================================================
``embed_joint``       DataEmbeddingLayer JOINT (+ static SUM_ALL, temporal encoding, NA level cumsum, mask):
                      data_embedding_layer.py:351-388, 609-708; transformer.py:594-672, 903-936
``embed_split_bags``  the two EmbeddingBag gathers of ``_split_embed`` (data_embedding_layer.py:390-450)
``embed_epilogue``    temporal encoding / level cumsum / mask after the SPLIT projection (the bf16 / f32 SPLIT
                      path runs ``split_proj_prep`` + GEMM + ``embed_epilogue`` in kernels._SplitProjection)
``attention``         InnerSelfAttention._attn (transformer.py:171-217) on a packed q|k|v buffer
``residual_ln``       residual + resid dropout + event mask + LayerNorm (transformer.py:350-461, 810-831)
``bias_act``          c_fc bias + activation (transformer.py:378-391)
``linear``            a bias-optional projection on the bf16 weight shadow, gradients to the f32 parameters
``mlp``               InnerMLP up to c_proj's bias (transformer.py:378-391)
``output_loss``       get_{classification,regression,TTE}_outputs + weighted_loss (model_output.py:1311-1721)
``head_loss``         the generative heads' GEMM + ``output_loss`` (model_output.py:1253-1721)
====================  =====================================================================================

``residual``          InnerBlock's last residual (+ the event-mask where of the NA glue; transformer.py:409-461)

Used by the NA glue's autograd Functions (transformer/structured_attention.py): ``na_split`` / ``na_split_bwd_``,
``na_assemble`` / ``na_assemble_bwd`` (structured_attention.py:63-156).

Non-differentiable: ``embed_bag_bwd``, ``embed_epilogue_bwd``, ``attention_bwd``, ``residual_ln_bwd``,
``bias_act_bwd``, ``linear_act``, ``linear_bwd`` (+ ``weight_grad_join``: with ``dw_tickets`` the weight gradient
runs on a second stream, joined by that op), ``gemm`` / ``gemm_``, ``column_sum``, ``kv_append``,
``attn_decode`` (generation), ``pack`` (the compute-dtype parameter copies) and ``adamw``
(generative_modeling.py:460-485).

There is no CPU kernel: calling an operator on CPU tensors raises (no fallback).
"""
from __future__ import annotations

import os

import torch

from . import _lib as L

_HERE = os.path.dirname(os.path.abspath(__file__))
TORCH_LIB_PATH = os.environ.get("ESGPT_AMD_TORCH_LIB", os.path.join(_HERE, "libesgpt_torch.so"))
ACT_DERIV = 8  # ESGPT_ACT_DERIV (include/esgpt_amd.h): the pre-activation buffer holds act'(pre)
_state = {"loaded": False}

OPS = ("embed_joint", "embed_split_bags", "embed_epilogue", "embed_epilogue_bwd", "embed_bag_bwd", "attention",
       "attention_bwd", "kv_append", "attn_decode", "output_loss", "residual_ln", "residual_ln_bwd", "bias_act",
       "bias_act_bwd", "column_sum", "gemm", "gemm_", "linear_act", "linear_bwd", "linear", "mlp", "head_loss",
       "pack", "adamw", "adamw_dev", "weight_grad_join", "residual_ln_bwd_partials", "colsum_flush", "seed_bank", "residual",
       "residual_bwd", "na_split", "na_split_bwd_", "na_assemble", "na_assemble_bwd", "na_head_split",
       "na_head_split_bwd", "split_proj_prep", "split_proj_post", "row_tiles")


def load():
    """Loads ``libesgpt_torch.so`` (once) and registers the fake kernels and autograd formulas; returns
    ``torch.ops.esgpt``. Raises ``HipExtensionMissing`` when the library has not been built."""
    if not _state["loaded"]:
        L.load(require_device=False)  # the kernel library first (libesgpt_torch.so links it by $ORIGIN)
        if not os.path.exists(TORCH_LIB_PATH):
            raise L.HipExtensionMissing(
                f"eventstreamgpt_amd: custom-op library not found at {TORCH_LIB_PATH}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C eventstreamgpt_amd/csrc`).")
        torch.ops.load_library(TORCH_LIB_PATH)
        _register()
        _state["loaded"] = True
    return torch.ops.esgpt


def _tickets(device):
    from .kernels import tickets

    return tickets(device)


def _leaves(*ts) -> bool:
    """Every gradient recipient is a leaf (a parameter): its gradient goes to AccumulateGrad, which steals it
    without a kernel — so a weight gradient still in flight on the weight-gradient stream is not read by the
    current stream before the join (TrainStep's parameter hooks join before any accumulation that would)."""
    return all(t is None or t.is_leaf for t in ts)


def _linear_bwd(dy, x, w, alpha, act, pre, need_dx, need_db, db_extra=None, split_ok=False, dw_out=None,
                db_out=None, row_tiles=None):
    """``esgpt::linear_bwd`` from a registered backward (records the launch shape for bench.py when asked). With
    ``split_ok`` (the weight / bias gradients go straight to leaf parameters) and inside ``weight_grad_overlap``,
    the weight gradient runs on the weight-gradient stream. ``dw_out`` / ``db_out`` (exchange-buffer regions,
    ``_dest``): the gradients are written there and returned as views of them."""
    from . import fused

    if fused.SHAPES["enabled"]:
        fused.SHAPES["linear_bwd"].append((dy.shape[0], x.shape[1], dy.shape[1], bool(need_dx), int(act),
                                           bool(need_db)))
    from .kernels import tickets, weight_grad_overlap_active

    dw_tickets = tickets(x.device, 1) if (split_ok and weight_grad_overlap_active(x.device)) else None
    dx, dw, db = torch.ops.esgpt.linear_bwd(dy, x, w, alpha, act, pre, need_dx, need_db, _tickets(x.device),
                                            db_extra, dw_tickets, dw_out, db_out if need_db else None, row_tiles)
    if dw_out is not None:
        dw = dw_out.view(dy.shape[1], x.shape[1])
    if need_db and db_out is not None:
        db = db_out
    return dx, dw, db


def _dest(ok: bool, tensors, pad: int = 0, shape=None):
    """The exchange-buffer region for the gradients of the leaf parameters ``tensors`` (kernels.grad_region; None
    when ``ok`` is False, e.g. a non-leaf recipient, or no destination is active), viewed as ``shape``."""
    if not ok:
        return None
    from .kernels import grad_region

    r = grad_region(tensors, pad)
    return r if (r is None or shape is None) else r.view(shape)


def _note(ok: bool, tensors, pad: int = 0):
    if ok:
        from .kernels import note_grad_group

        note_grad_group(tensors, pad)


def _tail(ctx, n: int) -> tuple:
    """Nones for the trailing optional arguments the caller passed explicitly: the backward returns one entry per
    argument of the call as dispatched (trailing arguments left at their defaults are not part of it), which is
    what ``ctx.needs_input_grad`` lists."""
    return (None,) * (len(ctx.needs_input_grad) - n)


def _batch_d(args, start):
    """(B, L, M) from the 9 batch tensors starting at args[start]."""
    di = args[start + 3]
    return di.shape[0], di.shape[1], di.shape[2]


def _register():
    lib = "esgpt::"
    fake = torch.library.register_fake
    E = torch.empty

    # ---------------------------------------------------------------- fake (meta) kernels
    @fake(lib + "embed_joint")
    def _(table, em, td, tm, di, dm, dv, dvm, si, sm, buckets, sin_div, cos_div, flags, static_w, dynamic_w, G, err):
        return table.new_empty(di.shape[0], di.shape[1], G, table.shape[1], dtype=torch.float32)

    @fake(lib + "embed_split_bags")
    def _(ct, nt, em, td, tm, di, dm, dv, dvm, si, sm, buckets, flags, cs, ns, ss, G, err):
        return ct.new_empty(di.shape[0] * di.shape[1] * G, ct.shape[1] + nt.shape[1], dtype=torch.float32)

    @fake(lib + "embed_epilogue")
    def _(y, em, td, tm, di, dm, dv, dvm, si, sm, G, flags, sin_div, cos_div):
        return y.new_empty(di.shape[0], di.shape[1], G, y.shape[-1], dtype=torch.float32)

    @fake(lib + "embed_epilogue_bwd")
    def _(dout, em, td, tm, di, dm, dv, dvm, si, sm, G, flags, dtype=None):
        return dout.new_empty(di.shape[0] * di.shape[1] * G, dout.shape[-1], dtype=dtype or torch.float32)

    @fake(lib + "split_proj_prep")
    def _(x, cat_w, num_w, cat_b, num_b, a_c, a_n, dtype):
        D, Dx = cat_w.shape[0], cat_w.shape[1] + num_w.shape[1]
        n = x.numel() // Dx if dtype == torch.bfloat16 else 0
        return (x.new_empty(n, Dx, dtype=dtype) if n else x.new_empty(0, dtype=torch.float32),
                x.new_empty(D, Dx, dtype=dtype), x.new_empty(D, dtype=torch.float32))

    @fake(lib + "split_proj_post")
    def _(dx_lp, dw, db, Dc, a_c, a_n, cat_dw, num_dw, cat_db, num_db):
        return dw.new_empty(0) if dx_lp is None else dw.new_empty(dx_lp.numel() // dw.shape[1], dw.shape[1])

    @fake(lib + "embed_bag_bwd")
    def _(dsrc, em, td, tm, di, dm, dv, dvm, si, sm, buckets, selector, flags, dyn_scale, static_scale, ld, D, V, G,
          out=None):
        return dsrc.new_empty(0 if out is not None else V, D, dtype=torch.float32)

    @fake(lib + "attention")
    def _(qkv, key_mask, query_mask, H, window, skf, p, seed):
        Bs, T, D3 = qkv.shape
        Lq = T - (1 if skf else 0)
        # keep bits: the MFMA path (bf16, hd in {16, 32, 64, 128}, Lk >= 16) with dropout (esgpt_attn_keep_words)
        hd = D3 // 3 // H
        nkeep = Bs * H * Lq * ((T + 31) // 32) if (p > 0 and qkv.dtype == torch.bfloat16 and hd in (16, 32, 64, 128)
                                                    and T >= 16) else 0
        return (qkv.new_empty(Bs, Lq, D3 // 3), qkv.new_empty(Bs, H, Lq, dtype=torch.float32),
                qkv.new_empty(nkeep, dtype=torch.int32))

    @fake(lib + "attention_bwd")
    def _(qkv, o, dout, lse, key_mask, query_mask, H, window, skf, p, seed, keep, tickets):
        return torch.empty_like(qkv)

    @fake(lib + "residual")
    def _(x, y, row_mask, mask_div, skip_T, p, seed):
        D = y.shape[-1]
        return y.new_empty(y.numel() // D, D, dtype=torch.float32)

    @fake(lib + "residual_bwd")
    def _(dh, row_mask, mask_div, skip_T, x_rows, need_dx, p, seed, y_dtype):
        D = dh.shape[-1]
        dx = dh.new_empty(x_rows, D, dtype=torch.float32) if need_dx else None
        return dx, dh.new_empty(dh.numel() // D, D, dtype=y_dtype)

    @fake(lib + "na_split")
    def _(x, event_mask):
        return x.new_empty(x.shape[0], x.shape[1], x.shape[3], dtype=torch.float32)

    @fake(lib + "na_split_bwd_")
    def _(dper, event_mask, dx):
        return None

    @fake(lib + "na_assemble")
    def _(ctx, x):
        B, L, G, D = x.shape
        return x.new_empty(B * L, G + 1, D, dtype=torch.float32)

    @fake(lib + "na_assemble_bwd")
    def _(dseq, B, L):
        G1, D = dseq.shape[-2], dseq.shape[-1]
        return dseq.new_empty(B, L, D, dtype=torch.float32), dseq.new_empty(B, L, G1 - 1, D, dtype=torch.float32)

    @fake(lib + "na_head_split")
    def _(x, dtype):
        B, L, G, D = x.shape
        return x.new_empty(B * L * (G - 1), D, dtype=dtype), x.new_empty(B * L, D, dtype=dtype)

    @fake(lib + "na_head_split_bwd")
    def _(dhead, dlast, B, L, G):
        g = dhead if dhead is not None else dlast
        return g.new_empty(B, L, G, g.shape[-1], dtype=torch.float32)

    @fake(lib + "kv_append")
    def _(qkv, k_cache, v_cache, past):
        return None

    @fake(lib + "attn_decode")
    def _(qkv, k_cache, v_cache, key_mask, query_mask, H, Lk, window):
        return qkv.new_empty(qkv.shape[0], qkv.shape[1], qkv.shape[2] // 3)

    def _loss_fake(zc, zt, shift, n_terms, B):
        f32 = torch.float32
        dzt = zc.new_empty(0) if zt is None else torch.empty_like(zt)
        dbias = zc.new_empty(B, zc.shape[-1], dtype=f32) if shift else zc.new_empty(0, dtype=f32)
        return zc.new_empty(n_terms + 2, dtype=f32), torch.empty_like(zc), dzt, dbias

    @fake(lib + "output_loss")
    def _(zc, zt, zc_bias, em, td, tm, di, dm, dv, dvm, si, sm, n_levels, shift, terms, tte_i, tte_f, err, path=0):
        return _loss_fake(zc, zt, shift, len(terms) // 8, di.shape[0])

    @fake(lib + "head_loss")
    def _(xc, xt, em, td, tm, di, dm, dv, dvm, si, sm, terms, tte_i, tte_f, shift, n_levels, wc, bc, wt, bt, cw, cb,
          tw, tb, err, tickets, zb):
        zc = xc.new_empty(xc.shape[0], wc.shape[0])
        zt = None if wt is None else xt.new_empty(xt.shape[0], wt.shape[0])
        return _loss_fake(zc, zt, shift, len(terms) // 8, di.shape[0])

    @fake(lib + "residual_ln")
    def _(x, y, bias, ln_w, ln_b, row_mask, p, seed, eps, out_dtype, skip_T=0):
        ref = y if y is not None else x  # the output rows (x holds more under skip_T)
        N, D = ref.shape
        f = ln_w.new_empty
        return f(N, D, dtype=torch.float32), f(N, D, dtype=out_dtype), f(N, dtype=torch.float32), \
            f(N, dtype=torch.float32)

    @fake(lib + "residual_ln_bwd")
    def _(dh, dout, h, mean, rstd, ln_w, row_mask, p, seed, need_dx, need_dy, y_dtype, out_dtype, tickets, skip_T=0):
        N, D = h.shape
        f = h.new_empty
        xN = N // (skip_T - 1) * skip_T if skip_T else N
        return (f(xN, D, dtype=torch.float32) if need_dx else f(0, dtype=torch.float32),
                f(N, D, dtype=y_dtype) if need_dy else f(0, dtype=y_dtype), f(3, D, dtype=torch.float32))

    @fake(lib + "bias_act")
    def _(f, bias, act):
        return torch.empty_like(f)

    @fake(lib + "bias_act_bwd")
    def _(dg, f, bias, act):
        return torch.empty_like(f), f.new_empty(f.shape[1], dtype=torch.float32)

    @fake(lib + "column_sum")
    def _(x):
        return x.new_empty(x.shape[1], dtype=torch.float32)

    @fake(lib + "gemm")
    def _(a_layout, a, lda, b_layout, b, ldb, M, N, K, bias, alpha, out_dtype, tickets):
        return a.new_empty(M, N, dtype=out_dtype)

    @fake(lib + "gemm_")
    def _(c, a_layout, a, lda, b_layout, b, ldb, M, N, K, bias, alpha, accumulate, tickets):
        return None

    @fake(lib + "linear_act")
    def _(x, w, bias, act):
        y = x.new_empty(x.shape[0], w.shape[0])
        return (x.new_empty(x.shape[0], w.shape[0]) if act >= 0 else x.new_empty(0)), y

    @fake(lib + "weight_grad_join")
    def _(like):
        return None

    @fake(lib + "seed_bank")
    def _(counter, bank, err=None):
        return None

    @fake(lib + "residual_ln_bwd_partials")
    def _(dh, dout, h, mean, rstd, ln_w, row_mask, p, seed, need_dx, need_dy, y_dtype, out_dtype, skip_T=0):
        N, D = h.shape
        f = h.new_empty
        from .kernels import _lib_partials

        xN = N // (skip_T - 1) * skip_T if skip_T else N
        return (f(xN, D, dtype=torch.float32) if need_dx else f(0, dtype=torch.float32),
                f(N, D, dtype=y_dtype) if need_dy else f(0, dtype=y_dtype),
                f(_lib_partials(N), 3 * D, dtype=torch.float32))

    @fake(lib + "colsum_flush")
    def _(parts, sums):
        return None

    @fake(lib + "linear_bwd")
    def _(dy, x, w, alpha, act, pre, need_dx, need_db, tickets, db_extra=None, dw_tickets=None, dw_out=None,
          db_out=None, row_tiles=None):
        f32 = torch.float32
        return (x.new_empty(dy.shape[0], x.shape[1], dtype=dy.dtype) if need_dx else x.new_empty(0, dtype=dy.dtype),
                x.new_empty(0, dtype=f32) if dw_out is not None else x.new_empty(dy.shape[1], x.shape[1], dtype=f32),
                x.new_empty(dy.shape[1], dtype=f32) if (need_db and db_out is None) else x.new_empty(0, dtype=f32))

    @fake(lib + "pack")
    def _(srcs, group_sizes, tails, dtypes):
        outs, k = [], 0
        for n_src, tail, code in zip(group_sizes, tails, dtypes):
            n = sum(t.numel() for t in srcs[k: k + n_src])
            k += n_src
            outs.append(srcs[0].new_empty(n + tail, dtype=torch.bfloat16 if code == L.BF16 else torch.float32))
        return outs

    @fake(lib + "linear")
    def _(x, w, bias, masters, tickets, row_tiles=None):
        return x.new_empty(x.shape[0], w.shape[0])

    @fake(lib + "row_tiles")
    def _(event_mask, rows_per_event):
        return event_mask.new_empty((event_mask.numel() * rows_per_event + 63) // 64, dtype=torch.uint8)

    @fake(lib + "mlp")
    def _(x, w_fc, w_pj, b_fc, b_pj, act, p_fc, p_pj, tickets, row_tiles=None):
        T = x.shape[0]
        return x.new_empty(T, w_pj.shape[0]), x.new_empty(T, w_fc.shape[0]), x.new_empty(T, w_fc.shape[0])

    @fake(lib + "adamw")
    def _(table, blocks, lr, beta1, beta2, eps, wd, step, per_tensor, err):
        return None

    @fake(lib + "adamw_dev")
    def _(table, blocks, counters, active, n_params, kind, warmup, total, power, init_lr, end_lr, beta1, beta2, eps,
          wd, per_tensor, lr_dev, err, copy_src=None, ring=None, ring_ctr=None, ring_tab=None, host_words=0):
        return None

    # ---------------------------------------------------------------- autograd formulas
    reg = torch.library.register_autograd
    ops = torch.ops.esgpt

    # embed_joint: d table (the EmbeddingBag backward, atomic-free CSR form; NA cumsum undone first)
    def _ej_setup(ctx, inputs, output):
        table, *batch = inputs[:10]
        buckets, sin_div, cos_div, flags, static_w, dynamic_w, G, err = inputs[10:]
        ctx.save_for_backward(*batch)
        ctx.meta = (tuple(buckets), flags, static_w, dynamic_w, G, table.shape[0], table.shape[1])
        ctx.table = table if table.is_leaf else None

    def _ej_bwd(ctx, dout):
        batch = ctx.saved_tensors
        buckets, flags, static_w, dynamic_w, G, V, D = ctx.meta
        dout = dout.contiguous().float()
        if flags & L.EMB_CUMSUM:
            dsrc = ops.embed_epilogue_bwd(dout, *batch, G, flags)
        else:
            dsrc = dout.view(-1, D)
        S = 0 if batch[7] is None else batch[7].shape[1]
        static = bool(flags & L.EMB_STATIC) and S > 0
        out = _dest(ctx.table is not None, [ctx.table])
        dtable = ops.embed_bag_bwd(dsrc, *batch, list(buckets), L.BAG_JOINT, flags,
                                   dynamic_w if static else 1.0, static_w, D, D, V, G, out)
        return (dtable if out is None else out.view(V, D),) + (None,) * 17

    reg(lib + "embed_joint", _ej_bwd, setup_context=_ej_setup)

    # embed_split_bags: d cat_table, d num_table (the two bag backwards over column blocks of dx)
    def _es_setup(ctx, inputs, output):
        ct, nt, *rest = inputs
        batch = rest[:9]
        buckets, flags, cat_scale, num_scale, static_scale, G, err = rest[9:]
        ctx.save_for_backward(*batch)
        ctx.meta = (tuple(buckets), flags, cat_scale, num_scale, static_scale, G, ct.shape[0], ct.shape[1],
                    nt.shape[1])
        ctx.tables = (ct, nt) if _leaves(ct, nt) else None

    def _es_bwd(ctx, dx):
        batch = ctx.saved_tensors
        buckets, flags, cat_scale, num_scale, static_scale, G, V, Dc, Dn = ctx.meta
        dx = dx.contiguous().float()
        if static_scale == 0.0:
            flags &= ~L.EMB_STATIC
        ok = ctx.tables is not None
        oc = _dest(ok, ctx.tables[:1] if ok else None)
        on = _dest(ok, ctx.tables[1:] if ok else None)
        dcat = ops.embed_bag_bwd(dx, *batch, list(buckets), L.BAG_CAT, flags, cat_scale, static_scale, Dc + Dn, Dc,
                                 V, G, oc)
        dnum = ops.embed_bag_bwd(dx[:, Dc:], *batch, list(buckets), L.BAG_NUM, flags, num_scale, 0.0, Dc + Dn, Dn,
                                 V, G, on)
        return (dcat if oc is None else oc.view(V, Dc), dnum if on is None else on.view(V, Dn)) + (None,) * 16

    reg(lib + "embed_split_bags", _es_bwd, setup_context=_es_setup)

    # embed_epilogue: d y
    def _ee_setup(ctx, inputs, output):
        y, *rest = inputs
        ctx.save_for_backward(*rest[:9])
        ctx.meta = (rest[9], rest[10], tuple(y.shape))

    def _ee_bwd(ctx, dout):
        G, flags, yshape = ctx.meta
        dy = ops.embed_epilogue_bwd(dout.contiguous().float(), *ctx.saved_tensors, G, flags)
        return (dy.view(yshape),) + (None,) * 13

    reg(lib + "embed_epilogue", _ee_bwd, setup_context=_ee_setup)

    # attention: d qkv (one fused MFMA backward reading the forward's dropout keep bits; the other paths regenerate
    # the keep mask from the same seed)
    def _at_setup(ctx, inputs, output):
        qkv, km, qm, H, window, skf, p, seed = inputs
        o, lse, keep = output
        ctx.mark_non_differentiable(lse, keep)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(qkv, o, lse, km, qm, seed, keep)
        ctx.meta = (H, window, skf, p)

    def _at_bwd(ctx, do, _dlse, _dkeep):
        if do is None:
            return (None,) * 8
        qkv, o, lse, km, qm, seed, keep = ctx.saved_tensors
        H, window, skf, p = ctx.meta
        dqkv = ops.attention_bwd(qkv, o, do, lse, km, qm, H, window, skf, p, seed, keep, _tickets(qkv.device))
        return dqkv, None, None, None, None, None, None, None

    reg(lib + "attention", _at_bwd, setup_context=_at_setup)

    # residual: d x (all rows of x; zeros for the rows skip_T leaves out), d y (y's dtype)
    def _rs_setup(ctx, inputs, output):
        x, y, row_mask, mask_div, skip_T, p, seed = inputs
        ctx.save_for_backward(row_mask, seed)
        ctx.meta = (mask_div, skip_T, 0 if x is None else x.numel() // x.shape[-1], p, y.dtype,
                    None if x is None else tuple(x.shape), tuple(y.shape))
        ctx.set_materialize_grads(False)

    def _rs_bwd(ctx, dh):
        if dh is None:
            return (None,) * 7
        row_mask, seed = ctx.saved_tensors
        mask_div, skip_T, x_rows, p, y_dtype, xs, ys = ctx.meta
        need_dx = xs is not None and ctx.needs_input_grad[0]
        dx, dy = ops.residual_bwd(dh, row_mask, mask_div, skip_T, x_rows, need_dx, p, seed, y_dtype)
        return (None if dx is None else dx.view(xs)), dy.view(ys), None, None, None, None, None

    reg(lib + "residual", _rs_bwd, setup_context=_rs_setup)

    # na_head_split: d x from both outputs' gradients in one pass
    def _hs_setup(ctx, inputs, output):
        x, dtype = inputs
        ctx.meta = tuple(x.shape)
        ctx.set_materialize_grads(False)

    def _hs_bwd(ctx, dhead, dlast):
        B, L, G, _ = ctx.meta
        if dhead is None and dlast is None:
            return None, None
        return ops.na_head_split_bwd(dhead, dlast, B, L, G), None

    reg(lib + "na_head_split", _hs_bwd, setup_context=_hs_setup)

    # residual_ln: d x, d y, d bias, d ln_w, d ln_b (column sums in the same launch)
    def _rl_setup(ctx, inputs, output):
        x, y, bias, ln_w, ln_b, row_mask, p, seed, eps, out_dtype, *rest = inputs
        skip_T = rest[0] if rest else 0
        h, out, mean, rstd = output
        ctx.mark_non_differentiable(mean, rstd)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(h, mean, rstd, ln_w, row_mask, seed)
        ctx.meta = (x is not None, y is not None, bias is not None, y.dtype if y is not None else torch.float32,
                    out_dtype, p, skip_T, len(inputs))
        ctx.defer_ok = bias is None and _leaves(ln_w, ln_b)
        # the deferred column sums [d ln_w | d ln_b | unused bias row] as one exchange-buffer region
        ctx.lnp = (ln_w, ln_b) if ctx.defer_ok else None
        _note(ctx.defer_ok, (ln_w, ln_b), ln_w.numel())

    def _rl_bwd(ctx, dh, dout, _dm, _dr):
        from .kernels import colsum_deferral_active, defer_colsum

        h, mean, rstd, ln_w, row_mask, seed = ctx.saved_tensors
        has_x, has_y, has_bias, y_dtype, out_dtype, p, skip_T, n_in = ctx.meta
        if dout is None:
            dout = torch.zeros(h.shape, dtype=out_dtype, device=h.device)
        if ctx.defer_ok and colsum_deferral_active(h.device):
            # partials now, the column sums in the pass's one esgpt::colsum_flush launch
            dx, dy, part = ops.residual_ln_bwd_partials(dh, dout, h, mean, rstd, ln_w, row_mask, p, seed, has_x,
                                                        has_y, y_dtype, out_dtype, skip_T)
            sums = _dest(True, ctx.lnp, h.shape[1], (3, h.shape[1]))
            if sums is None:
                sums = torch.empty(3, h.shape[1], dtype=torch.float32, device=h.device)
            defer_colsum(h.device, part, sums.view(-1))
        else:
            dx, dy, sums = ops.residual_ln_bwd(dh, dout, h, mean, rstd, ln_w, row_mask, p, seed, has_x, has_y,
                                               y_dtype, out_dtype, _tickets(h.device), skip_T)
        return (dx if has_x else None, dy if has_y else None, sums[2] if has_bias else None, sums[0], sums[1],
                None, None, None, None, None) + (None,) * (n_in - 10)

    reg(lib + "residual_ln", _rl_bwd, setup_context=_rl_setup)

    # bias_act: d f, d bias
    def _ba_setup(ctx, inputs, output):
        f, bias, act = inputs
        ctx.save_for_backward(f, bias)
        ctx.act = act

    def _ba_bwd(ctx, dg):
        f, bias = ctx.saved_tensors
        dz, dbias = ops.bias_act_bwd(dg, f, bias, ctx.act)
        return dz, dbias, None

    reg(lib + "bias_act", _ba_bwd, setup_context=_ba_setup)

    # linear: d x, d bias, and the f32 weight gradient split over the master parameters (one grouped launch)
    def _li_setup(ctx, inputs, output):
        x, w, bias, masters, tickets, *rest = inputs
        ctx.row_tiles = rest[0] if rest else None  # padded-event row blocks: the dX product skips them too
        ctx.save_for_backward(x, w)
        ctx.rows = [m.shape[0] for m in masters]
        ctx.has_bias = bias is not None
        ctx.split_ok = _leaves(bias, *masters)
        ctx.gp = (list(masters), bias) if ctx.split_ok and masters else None
        _note(ctx.gp is not None and len(masters) > 1, masters)

    def _li_bwd(ctx, dy):
        x, w = ctx.saved_tensors
        need_db = ctx.has_bias and ctx.needs_input_grad[2]
        ok = ctx.gp is not None
        dw_out = _dest(ok, ctx.gp[0] if ok else None)
        db_out = _dest(ok and need_db, [ctx.gp[1]] if ok else None)
        dx, dw, db = _linear_bwd(dy, x, w, None, -1, None, ctx.needs_input_grad[0], need_db, split_ok=ctx.split_ok,
                                 dw_out=dw_out, db_out=db_out, row_tiles=ctx.row_tiles)
        return (dx if ctx.needs_input_grad[0] else None, None, db if need_db else None,
                list(torch.split(dw, ctx.rows, 0)), None) + _tail(ctx, 5)

    reg(lib + "linear", _li_bwd, setup_context=_li_setup)

    # mlp: d x, d b_fc, d b_proj, d W_fc, d W_proj (activation gradient in c_proj's dX epilogue, the bias gradients
    # as row sums inside the dW products)
    def _ml_setup(ctx, inputs, output):
        x, w_fc, w_pj, b_fc, b_pj, act, p_fc, p_pj, tickets, *rest = inputs
        ctx.row_tiles = rest[0] if rest else None
        y, pre, g = output
        ctx.mark_non_differentiable(pre, g)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, w_fc, w_pj, pre, g)
        ctx.act = act
        ctx.has_bpj = b_pj is not None
        ctx.split_ok = _leaves(b_fc, b_pj, p_fc, p_pj)
        ctx.gp = (p_fc, p_pj, b_fc, b_pj) if ctx.split_ok else None

    def _ml_bwd(ctx, dy, _dpre, _dg):
        if dy is None:
            return (None,) * 9 + _tail(ctx, 9)
        x, w_fc, w_pj, pre, g = ctx.saved_tensors
        need_dbpj = ctx.has_bpj and ctx.needs_input_grad[4]
        ok = ctx.gp is not None
        gp = ctx.gp if ok else (None,) * 4
        # `pre` holds act'(pre-activation) (esgpt::mlp stores it with ESGPT_ACT_DERIV): the dX epilogue multiplies
        dz, dw_pj, db_pj = _linear_bwd(dy, g, w_pj, None, ctx.act | ACT_DERIV, pre, True, need_dbpj, split_ok=ctx.split_ok,
                                       dw_out=_dest(ok, [gp[1]]), db_out=_dest(ok and need_dbpj, [gp[3]]),
                                       row_tiles=ctx.row_tiles)
        need_dx = ctx.needs_input_grad[0]
        dx, dw_fc, db_fc = _linear_bwd(dz, x, w_fc, None, -1, None, need_dx, True, split_ok=ctx.split_ok,
                                       dw_out=_dest(ok, [gp[0]]), db_out=_dest(ok, [gp[2]]), row_tiles=ctx.row_tiles)
        return (dx if need_dx else None, None, None, db_fc, db_pj if need_dbpj else None, None, dw_fc, dw_pj,
                None) + _tail(ctx, 9)

    reg(lib + "mlp", _ml_bwd, setup_context=_ml_setup)

    # output_loss: d zc, d zt, d zc_bias (per-term entries of the losses output are for logging only)
    def _ol_setup(ctx, inputs, output):
        zc, zt, zc_bias = inputs[:3]
        losses, dzc, dzt, dbias = output
        ctx.mark_non_differentiable(dzc, dzt, dbias)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(dzc, dzt, dbias)
        ctx.meta = (zt is not None, zc_bias is not None)

    def _ol_bwd(ctx, g, *_):
        if g is None:
            return (None,) * 19
        dzc, dzt, dbias = ctx.saved_tensors
        has_zt, has_bias = ctx.meta
        gt = g[-1]
        d_bias = (dbias.sum(0) * gt).to(dzc.dtype) if (has_bias and dbias.numel()) else None
        return ((dzc * gt.to(dzc.dtype)), (dzt * gt.to(dzt.dtype)) if has_zt else None, d_bias) + (None,) * 16

    reg(lib + "output_loss", _ol_bwd, setup_context=_ol_setup)

    # head_loss: head GEMM backward scaled by d(total) read from device memory (the GEMM's alpha pointer)
    def _hl_setup(ctx, inputs, output):
        xc, xt = inputs[0], inputs[1]
        wc, bc, wt, bt, cw, cb, tw, tb = inputs[16:24]
        losses, dzc, dzt, dbias = output
        ctx.mark_non_differentiable(dzc, dzt, dbias)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(xc, xt, wc, wt, dzc, dzt, dbias)
        ctx.rows = ([w.shape[0] for w in cw], [w.shape[0] for w in tw])
        ctx.n = (len(cw), len(tw))
        ctx.split_ok = _leaves(*cw, *cb, *tw, *tb)
        # the padded head GEMM's dW / db rows [params | pad] as exchange-buffer regions
        D = xc.shape[1]
        pc = wc.shape[0] - sum(ctx.rows[0])
        pt = (wt.shape[0] - sum(ctx.rows[1])) if tw else 0
        ctx.gp = (list(cw), list(cb), list(tw), list(tb), pc, pt, D) if ctx.split_ok else None
        if ctx.gp is not None:
            _note(True, cw, pc * D)
            _note(True, cb, pc)
            if tw:
                _note(True, tw, pt * D)
                _note(True, tb, pt)

    def _hl_bwd(ctx, g, *_):
        if g is None:
            return (None,) * 27
        xc, xt, wc, wt, dzc, dzt, dbias = ctx.saved_tensors
        n_cw, n_tw = ctx.n
        rows_c, rows_t = ctx.rows
        alpha = g[-1:]  # a 1-element view (g may be a stride-0 expansion of the total's gradient)
        # the loss kernel's per-subject position-0 bias rows are summed into db inside the same launch
        gp = ctx.gp
        ok = gp is not None
        dxc, dwc, dbc = _linear_bwd(dzc, xc, wc, alpha, -1, None, True, True, dbias if dbias.numel() else None,
                                    split_ok=ctx.split_ok, dw_out=_dest(ok, gp and gp[0], gp and gp[4] * gp[6]),
                                    db_out=_dest(ok, gp and gp[1], gp and gp[4]))
        nc = sum(rows_c)
        gw_c = list(torch.split(dwc[:nc], rows_c, 0))
        gb_c = list(torch.split(dbc[:nc], rows_c, 0))
        dxt, gw_t, gb_t = None, [], []
        if n_tw:
            dxt, dwt, dbt = _linear_bwd(dzt, xt, wt, alpha, -1, None, True, True, split_ok=ctx.split_ok,
                                        dw_out=_dest(ok, gp and gp[2], gp and gp[5] * gp[6]),
                                        db_out=_dest(ok, gp and gp[3], gp and gp[5]))
            nt = sum(rows_t)
            gw_t = list(torch.split(dwt[:nt], rows_t, 0))
            gb_t = list(torch.split(dbt[:nt], rows_t, 0))
        return (dxc, dxt) + (None,) * 14 + (None, None, None, None, gw_c, gb_c, gw_t, gb_t,
                                             None, None, None)

    reg(lib + "head_loss", _hl_bwd, setup_context=_hl_setup)
