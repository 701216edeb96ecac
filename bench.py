"""Headline benchmark: CI-PPT training throughput (train events/sec) — BASELINE.json ``metric`` on ``configs[1]``
(C2: CI-PPT, 6 layers, d=256, L=256, global attention, synthetic EHR-shaped batches, one MI355X per rank).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-graph] [--no-cpu-baseline]
                    [--roofline-only] [--no-roofline]

A step = the batch's copy into the step graph's input buffer + forward + backward + (RCCL gradient
all-reduce, overlapped with backward) + AdamW + LR-schedule step on B=32 subjects per GPU (weak scaling); the timed
batches start in pinned host memory and each step's H2D (one copy of a packed batch, issued on a copy stream during
the previous step and waited on by the step) is inside the timed region. ``value_hbm_resident`` times the same step on
batches already resident in HBM (``--no-hbm-line`` skips it). ``--gpus N`` without torchrun's environment re-launches this script
under ``torch.distributed.run`` with N ranks (before any GPU call) and exits with its status. Rank 0 prints ONE
JSON line: ``value`` = events of all ranks / wall time of the K timed steps (max over ranks, barrier +
synchronize on both sides); ``ms_per_step_median`` = the median step time from HIP events between steps.

Also reported (rank 0):
* ``roofline``: the step's dominant kernel by device time, the grouped projection backward (dX + dW + db of one
  Linear in one launch, MFMA-bound, 4·T·in·out algorithmic FLOPs) over EVERY launch shape of one step (shapes
  recorded from a real step, each launch captured 20 times into a HIP graph and replayed between HIP events on the
  capturing stream, FLOP-weighted): ``frac`` is that step average; ``frac_isolated`` is c_fc's launch alone.
* ``roofline_aux``: the same measurement, at the configuration's own shapes, for the attention forward / backward
  (4·H·hd·T / 8·H·hd·T, T = allowed (query, key) pairs of the batch; the symbol is the kernel the
  library's dispatch launches, esgpt_attn_path), the c_fc forward, the input layer (JOINT, or the NA SPLIT bags) and
  its table-gradient backward (HBM bytes, §8d per-occurrence accounting), the fused output losses (CI, or the NA
  per-level rows), the §8d C5 embed-bag microbench over a bf16 table larger than the Infinity Cache (C2 / C5), a
  long-sequence attention forward and backward and the generation decode kernel.
* ``traffic`` (every entry) = HBM bytes per launch set from this configuration's own rocprofv3 PMC passes
  (profiles/pmc_traffic_<config>.json: FETCH_SIZE doubled per the gfx950 calibration + WRITE_SIZE; tools/pmc_traffic.py
  --entries over ``--roofline-only --pmc-pass``), null without one; HBM-bound entries also carry the counter bytes
  over the launch time (``achieved_counter_GBs``).
* ``cpu_baseline``: the f32 oracle port timed on this host's cores on a bounded sample of the same workload.
``--roofline-only`` runs just the roofline launches (the command the PMC passes profile).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from eventstreamgpt_amd.data.types import PytorchBatch  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.train import TrainStep, init_distributed  # noqa: E402
from eventstreamgpt_amd.transformer.config import OptimizationConfig  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def attention_flops_fwd(batch, cfg) -> float:
    """Algorithmic forward FLOPs per layer: 4 * H * hd * T, T = allowed (q, k) pairs over valid
    queries (causal: keys j <= i that are valid; local: also i - j < window)."""
    em = batch.event_mask.cpu()
    H, hd = cfg.num_attention_heads, cfg.head_dim
    cum = em.long().cumsum(1)
    T_glob = float((cum * em).sum())  # for each valid query: number of valid keys j <= i (global layers)
    return 4.0 * H * hd * T_glob


def embed_fwd_bytes(batch, cfg) -> float:
    """Algorithmic bytes of the JOINT input-layer kernel: gathered rows per occurrence + entries +
    output + static rows (gathered per event) + time/mask."""
    em = batch.event_mask.cpu()
    idx = batch.dynamic_indices.cpu()
    D = cfg.hidden_size
    valid = em.unsqueeze(-1) & (idx > 0)
    nnz = float(valid.sum())
    B, L, M = idx.shape
    S = batch.static_indices.shape[1]
    n_ev = float(em.sum())
    return nnz * D * 4 + B * L * M * 21 + B * L * D * 4 + n_ev * S * D * 4 + B * L * 5


def graph_time_ms(fn, reps: int = 20, iters: int = 5) -> float:
    """Average device time of one ``fn()`` launch: ``reps`` launches captured into one HIP graph, the graph replayed
    ``iters`` times between HIP events on the current (replaying) stream."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * iters)


def _attention_launchers(B, Lq, D, H, em, p, dev, dtype=torch.bfloat16):
    """esgpt_attn_fwd_ex / esgpt_attn_bwd_ex launches on preallocated packed-qkv buffers (the step's layout and
    path: the forward writes the dropout keep bits the backward reads, as the attention operator does), in the
    step's compute dtype (bf16, or f32: the reference-precision kernels)."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import tickets

    lib = L.load()
    hd = D // H
    code = L.BF16 if dtype == torch.bfloat16 else L.F32
    g = torch.Generator(device=dev).manual_seed(0)
    bufs = {"qkv": (0.5 * torch.randn(B, Lq, 3 * D, device=dev, generator=g)).to(dtype),
            "o": torch.empty(B, Lq, D, device=dev, dtype=dtype),
            "lse": torch.empty(B, H, Lq, device=dev),
            "do": torch.randn(B, Lq, D, device=dev, generator=g).to(dtype),
            "seed": torch.tensor([12345], dtype=torch.int64, device=dev),
            "em": em.to(torch.bool).contiguous()}
    bufs["dqkv"] = torch.empty_like(bufs["qkv"])
    nbytes = lib.esgpt_attn_bwd_workspace(B, H, Lq, Lq, hd)
    bufs["ws"] = torch.empty(max(1, nbytes), dtype=torch.uint8, device=dev)
    nkeep = lib.esgpt_attn_keep_words(B, H, Lq, Lq, hd, Lq, 3 * D, D, code, p)
    bufs["keep"] = torch.empty(max(1, nkeep), dtype=torch.int32, device=dev)
    kp = bufs["keep"].data_ptr() if nkeep else None
    es = bufs["qkv"].element_size()
    base, dbase, m = bufs["qkv"].data_ptr(), bufs["dqkv"].data_ptr(), bufs["em"].data_ptr()
    cnt = tickets(torch.device(dev))

    def fwd():
        L.check(lib.esgpt_attn_fwd_ex(base, base + D * es, base + 2 * D * es, 3 * D, Lq, bufs["o"].data_ptr(), D,
                                      bufs["lse"].data_ptr(), m, m, B, H, Lq, Lq, hd, 0, p, bufs["seed"].data_ptr(),
                                      code, kp, L.stream()), "attn_fwd")

    def bwd():
        L.check(lib.esgpt_attn_bwd_ex(base, base + D * es, base + 2 * D * es, 3 * D, Lq, bufs["o"].data_ptr(), D,
                                      bufs["do"].data_ptr(), D, bufs["lse"].data_ptr(), m, m, dbase, dbase + D * es,
                                      dbase + 2 * D * es, 3 * D, B, H, Lq, Lq, hd, 0, p, bufs["seed"].data_ptr(), kp,
                                      code, bufs["ws"].data_ptr(), nbytes, cnt.data_ptr(), L.stream()), "attn_bwd")

    fwd()
    return fwd, bwd, bufs, cnt


def _gemm_launchers(T, D, F, dev, dtype=torch.bfloat16):
    """c_fc on the step's shapes: forward with the bias + GELU epilogue, and its grouped backward (bf16 MFMA, or the
    exact-f32 MFMA kernels of the reference-precision step)."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import tickets

    lib = L.load()
    f32 = dtype == torch.float32
    g = torch.Generator(device=dev).manual_seed(1)
    bufs = {"x": torch.randn(T, D, device=dev, generator=g).to(dtype),
            "w": (0.05 * torch.randn(F, D, device=dev, generator=g)).to(dtype),
            "b": torch.zeros(F, device=dev), "pre": torch.empty(T, F, device=dev, dtype=dtype),
            "y": torch.empty(T, F, device=dev, dtype=dtype),
            "dy": torch.randn(T, F, device=dev, generator=g).to(dtype),
            "dx": torch.empty(T, D, device=dev, dtype=dtype),
            "dw": torch.empty(F, D, device=dev), "db": torch.empty(F, device=dev)}
    nb = (lib.esgpt_linear_bwd_f32_workspace if f32 else lib.esgpt_linear_bwd_workspace)(T, D, F, 1)
    bufs["ws"] = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
    cnt = tickets(torch.device(dev))
    P = {k: v.data_ptr() for k, v in bufs.items()}

    def fwd():
        L.check((lib.esgpt_linear_fwd_f32 if f32 else lib.esgpt_linear_fwd)(P["x"], D, P["w"], T, D, F, P["b"], 0,
                                                                            P["pre"], P["y"], F, L.stream()),
                "linear_fwd")

    def bwd():
        if f32:
            L.check(lib.esgpt_linear_bwd_f32(P["dy"], F, P["x"], D, P["w"], T, D, F, None, -1, None, 0, P["dx"], D,
                                             P["dw"], P["db"], P["ws"], nb, cnt.data_ptr(), None, 0, L.stream()),
                    "linear_bwd_f32")
        else:
            L.check(lib.esgpt_linear_bwd(P["dy"], F, P["x"], D, P["w"], T, D, F, None, -1, None, 0, P["dx"], D,
                                         P["dw"], P["db"], P["ws"], nb, cnt.data_ptr(), L.stream()), "linear_bwd")

    return fwd, bwd, bufs


def _decode_launcher(B, H, hd, Lk, dev):
    """esgpt_attn_decode for one generated event per subject over a cache of Lk events (f32, the generation dtype):
    HBM-bound, algorithmic bytes = B·H·Lk·hd·4·2 (every cached key and value row once) + q and o rows."""
    from eventstreamgpt_amd import _lib as L

    lib = L.load()
    D = H * hd
    g = torch.Generator(device=dev).manual_seed(2)
    bufs = {"qkv": torch.randn(B, 1, 3 * D, device=dev, generator=g),
            "k": torch.randn(B, Lk, D, device=dev, generator=g), "v": torch.randn(B, Lk, D, device=dev, generator=g),
            "o": torch.empty(B, 1, D, device=dev)}
    P = {k: v.data_ptr() for k, v in bufs.items()}

    def fwd():
        L.check(lib.esgpt_attn_decode(P["qkv"], 3 * D, P["k"], P["v"], None, None, P["o"], D, B, H, 1, Lk, Lk, hd, 0,
                                      L.F32, L.stream()), "attn_decode")

    return fwd, float(B * H * Lk * hd * 4 * 2 + 2 * B * D * 4), bufs


def embed_bwd_bytes(batch, cfg) -> float:
    """§8d embed-bag backward bytes: a gradient row read per occurrence (nnz·D·4) + index / weight per occurrence
    (8 + 4) + the table gradient written (V·D·4) + static rows (per event: the subject-summed gradient)."""
    em = batch.event_mask.cpu()
    idx = batch.dynamic_indices.cpu()
    D, V = cfg.hidden_size, cfg.vocab_size
    nnz = float((em.unsqueeze(-1) & (idx > 0)).sum())
    S = batch.static_indices.shape[1]
    return nnz * D * 4 + nnz * 12 + V * D * 4 + float(em.sum()) * D * 4 + batch.event_mask.shape[0] * S * (D * 4 + 12)


def _embed_bwd_launcher(model, batch):
    """The JOINT input layer's table gradient (esgpt_embed_bag_bwd: every kernel of the CSR-transpose backward)."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import bag_bwd

    emb = model.encoder.input_layer.data_embedding_layer
    B, Lq = batch.event_mask.shape
    D, V = emb.embed_layer.weight.shape[1], emb.embed_layer.weight.shape[0]
    g = torch.Generator(device=batch.device).manual_seed(3)
    dsrc = torch.randn(B * Lq, D, device=batch.device, generator=g)
    flags = emb._flags()
    static = bool(flags & L.EMB_STATIC) and batch.static_indices is not None and batch.static_indices.shape[1] > 0
    keep = {"dsrc": dsrc}

    def bwd():
        keep["out"] = bag_bwd(batch, emb._buckets, L.BAG_JOINT, flags, emb.dynamic_weight if static else 1.0,
                              emb.static_weight, dsrc, D, D, V, 1)

    return bwd, keep


def _loss_launcher(model, batch, dtype=torch.bfloat16):
    """esgpt_output_loss on the step's head layout (bf16 logits [B·L, C], every C2 loss term + TTE): count, event
    and reduce kernels. Algorithmic bytes: logits read + d(logits) written (C·2 each per row) + the batch's entries
    (idx 8 + meas 8 + value 4 + mask 1 per slot) + event mask / time delta + the position-0 bias-gradient rows."""
    import ctypes

    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import batch_view, err_word
    from eventstreamgpt_amd.transformer import model_output as MO

    layer = model.output_layer
    if layer._layout is None:
        layer._layout = layer._build_layout()
    terms, _ = layer._terms_for(MO.all_classification_measurements(layer),
                                MO.all_regression_measurements(layer.config), 0)
    tte = layer._tte_spec(layer._layout["n_content"])
    lib = L.load()
    bv = batch_view(batch)
    B, Lq, M = bv.B, bv.L, bv.M
    C = layer._layout["n_content"] + tte.K * (1 if tte.kind == L.TTE_EXP else 3)
    C += (-C) % 8
    dev = batch.device
    g = torch.Generator(device=dev).manual_seed(4)
    zc = torch.randn(B * Lq, C, device=dev, generator=g).to(dtype)
    bias = torch.zeros(C, device=dev).to(dtype)
    code, es = (L.BF16, 2) if dtype == torch.bfloat16 else (L.F32, 4)
    dzc = torch.empty_like(zc)
    dbias = torch.empty(B, C, device=dev)
    losses = torch.empty(len(terms) + 2, device=dev)
    nb = lib.esgpt_output_loss_workspace(B, Lq, len(terms))
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
    arr = (L.EsgptLossTerm * max(1, len(terms)))(*terms)
    err = err_word(dev)

    def fwd():
        L.check(lib.esgpt_output_loss(bv.ref, zc.data_ptr(), C, 1, 1, bias.data_ptr(), zc.data_ptr(), C, code, arr,
                                      len(terms), ctypes.byref(tte), dzc.data_ptr(), dzc.data_ptr(),
                                      dbias.data_ptr(), losses.data_ptr(), ws.data_ptr(), nb, err.data_ptr(),
                                      L.stream()), "output_loss")

    nbytes = B * Lq * C * es * 2 + B * Lq * M * 21 + B * Lq * 5 + B * C * 4
    return fwd, float(nbytes), {"zc": zc, "dzc": dzc, "ws": ws, "arr": arr, "tte": tte}


def gemm_bwd_in_step(model, opt_cfg, batch, dtype) -> dict:
    """The grouped projection backward over every launch shape of one training step: the shapes are recorded from
    a real (eager) step, each distinct shape is timed in isolation (graph of 20 launches), and the in-step rate is
    Σ count·FLOPs / Σ count·time."""
    from collections import Counter

    from eventstreamgpt_amd import fused
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import tickets
    from eventstreamgpt_amd.train import TrainStep

    ts = TrainStep(model, opt_cfg, compute_dtype=dtype, use_graph=False, check_errors=False)
    f32 = dtype == torch.float32
    fused.SHAPES["linear_bwd"].clear()
    fused.SHAPES["enabled"] = True
    try:
        ts.opt.zero_grad()
        ts._fwd_bwd(batch)
    finally:
        fused.SHAPES["enabled"] = False
    for p in model.parameters():
        p.grad = None
    shapes = Counter(fused.SHAPES["linear_bwd"])
    lib = L.load()
    dev = batch.device
    cnt = tickets(dev)
    tot_flops = tot_ms = 0.0
    rows = []
    for (T, din, dout, need_dx, act, need_db), n in sorted(shapes.items()):
        g = torch.Generator(device=dev).manual_seed(T + din + dout)
        dy = torch.randn(T, dout, device=dev, generator=g).to(dtype)
        x = torch.randn(T, din, device=dev, generator=g).to(dtype)
        w = torch.randn(dout, din, device=dev, generator=g).to(dtype)
        pre = torch.randn(T, din, device=dev, generator=g).to(dtype) if act >= 0 else None
        dx = torch.empty(T, din, device=dev, dtype=dtype) if need_dx else None
        dw = torch.empty(dout, din, device=dev)
        db = torch.empty(dout, device=dev) if need_db else None
        nb = (lib.esgpt_linear_bwd_f32_workspace if f32 else lib.esgpt_linear_bwd_workspace)(T, din, dout, int(need_dx))
        ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)

        def fn(dy=dy, x=x, w=w, pre=pre, dx=dx, dw=dw, db=db, ws=ws, nb=nb, T=T, din=din, dout=dout, act=act):
            if f32:  # the reference-precision step's kernel (exact-f32 MFMA)
                L.check(lib.esgpt_linear_bwd_f32(dy.data_ptr(), dout, x.data_ptr(), din, w.data_ptr(), T, din, dout,
                                                 None, act, L.ptr(pre), din if pre is not None else 0, L.ptr(dx),
                                                 din if dx is not None else 0, dw.data_ptr(), L.ptr(db),
                                                 ws.data_ptr(), nb, cnt.data_ptr(), None, 0, L.stream()),
                        "linear_bwd_f32")
            else:
                L.check(lib.esgpt_linear_bwd(dy.data_ptr(), dout, x.data_ptr(), din, w.data_ptr(), T, din, dout, None,
                                             act, L.ptr(pre), din if pre is not None else 0, L.ptr(dx),
                                             din if dx is not None else 0, dw.data_ptr(), L.ptr(db), ws.data_ptr(), nb,
                                             cnt.data_ptr(), L.stream()), "linear_bwd")

        ms = graph_time_ms(fn)
        flops = 2.0 * T * din * dout * (2 if need_dx else 1)
        tot_flops += n * flops
        tot_ms += n * ms
        rows.append({"T": T, "in": din, "out": dout, "dx": need_dx, "launches": n, "avg_ms": round(ms, 5),
                     "tflops": round(flops / (ms * 1e-3) / 1e12, 1)})
    return {"achieved": tot_flops / (tot_ms * 1e-3) / 1e12, "launches_per_step": sum(shapes.values()),
            "ms_per_step": tot_ms, "shapes": rows}


def _attn_symbol(lib, fwd: bool, hd: int, Lq: int, Lk: int, ld_in: int, ld_o: int, drop: bool,
                 dtype=torch.bfloat16, bh: int = 0) -> str:
    """The kernel esgpt_attn_fwd / _bwd actually launches for these arguments (the library's own dispatch rule;
    ``bh`` = batch x heads, for the forward's wide-form rule)."""
    from eventstreamgpt_amd import _lib as L

    path = lib.esgpt_attn_path(hd, Lq, Lk, Lq, ld_in, ld_o, L.BF16 if dtype == torch.bfloat16 else L.F32)
    d = "true" if drop else "false"
    if path == 1:
        # attention_mfma.hip fwd_wide_nw, attention_bwd.hip split2_keys
        if fwd and hd == 64 and Lq >= 512 and -(-Lq // 128) * bh >= 1024:
            return f"attn_fwd_wide_kernel<{hd}, {d}, 4 waves>"
        if not fwd and ((Lk > 256 and hd == 16) or (Lk >= 2048 and hd == 64 and not drop) or hd == 128):
            return f"attn_bwd_dkv_kernel<{hd}> + attn_bwd_dq_kernel<{hd}>"
        return f"attn_fwd_mfma_kernel<{hd}, {d}>" if fwd else f"attn_bwd_kernel<{hd}, {d}>"
    if path == 3:
        return (f"attn_fwd_f32_kernel<{hd}, {d}>" if fwd
                else f"attn_dq_f32_kernel<{hd}, {d}> + attn_dkv_f32_kernel<{hd}, {d}>")
    if path == 2:
        return "attn_fwd_small<bf16>" if fwd else "attn_bwd_small<bf16>"
    return "attn_fwd_generic<bf16>" if fwd else "attn_bwd_dq_generic<bf16> + attn_bwd_dkv_generic<bf16>"


def _na_loss_launcher(model, batch):
    """esgpt_output_loss on the NA head layout (per-level rows [B·L·(G-1), C], separate TTE rows [B·L, ldt]):
    algorithmic bytes = the level rows' logits read + gradients written, the TTE rows likewise, the entries."""
    import ctypes

    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import batch_view, err_word
    from eventstreamgpt_amd.transformer import model_output as MO

    layer = model.output_layer
    if layer._layout is None:
        layer._layout = layer._build_layout()
    c = model.config
    G = len(c.measurements_per_dep_graph_level)
    cls_all, reg_all = MO.all_classification_measurements(layer), MO.all_regression_measurements(c)
    terms = []
    for i in range(1, G):
        cat, num = MO._level_sets(c.measurements_per_dep_graph_level[i])
        terms += layer._terms_for(cat & cls_all, num & reg_all, i - 1)[0]
    tte = layer._tte_spec(0)
    lib = L.load()
    bv = batch_view(batch)
    B, Lq, M = bv.B, bv.L, bv.M
    C = layer._layout["n_content"]
    C += (-C) % 8
    ldt = 1 if tte.kind == L.TTE_EXP else 3 * tte.K
    dev = batch.device
    g = torch.Generator(device=dev).manual_seed(5)
    zc = torch.randn(B * Lq * (G - 1), C, device=dev, generator=g).bfloat16()
    zt = torch.randn(B * Lq, ldt, device=dev, generator=g).bfloat16()
    dzc, dzt = torch.empty_like(zc), torch.empty_like(zt)
    losses = torch.empty(len(terms) + 2, device=dev)
    nb = lib.esgpt_output_loss_workspace(B, Lq, len(terms))
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
    arr = (L.EsgptLossTerm * max(1, len(terms)))(*terms)
    err = err_word(dev)

    def fwd():
        L.check(lib.esgpt_output_loss(bv.ref, zc.data_ptr(), C, G - 1, 0, None, zt.data_ptr(), ldt, L.BF16, arr,
                                      len(terms), ctypes.byref(tte), dzc.data_ptr(), dzt.data_ptr(), None,
                                      losses.data_ptr(), ws.data_ptr(), nb, err.data_ptr(), L.stream()), "na_loss")

    nbytes = B * Lq * (G - 1) * C * 2 * 2 + B * Lq * ldt * 2 * 2 + B * Lq * M * 21 + B * Lq * 5
    return fwd, float(nbytes), {"zc": zc, "zt": zt, "dzc": dzc, "dzt": dzt, "ws": ws, "arr": arr, "tte": tte}


def _split_embed_launchers(model, batch):
    """NA SPLIT input layer (esgpt_embed_split_bags_fwd: both tables' bags for every (event, bucket)) and its two
    table-gradient backwards (categorical / numerical selectors)."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import EmbedSpec, bag_bwd, split_bags

    emb = model.encoder.input_layer.data_embedding_layer
    flags = emb._flags()
    G = emb.n_levels
    static = bool(flags & L.EMB_STATIC)
    dw = emb.dynamic_weight if static else 1.0
    cs, ns, ss = dw * emb.categorical_weight, dw * emb.numerical_weight, (emb.static_weight if static else 0.0)
    spec = EmbedSpec(flags, emb.static_weight, emb.dynamic_weight, emb._buckets, G)
    ct, nt = emb.categorical_embed_layer.weight, emb.numerical_embed_layer.weight
    V, Dc, Dn = ct.shape[0], ct.shape[1], nt.shape[1]
    B, Lq = batch.event_mask.shape
    keep = {"dx": torch.randn(B * Lq * G, Dc + Dn, device=batch.device,
                              generator=torch.Generator(device=batch.device).manual_seed(6))}

    def fwd():
        with torch.no_grad():
            keep["x"] = split_bags(ct, nt, batch, spec, cs, ns, ss)

    def bwd():
        keep["dc"] = bag_bwd(batch, emb._buckets, L.BAG_CAT, flags, cs, ss, keep["dx"], Dc + Dn, Dc, V, G)
        keep["dn"] = bag_bwd(batch, emb._buckets, L.BAG_NUM, flags & ~L.EMB_STATIC, ns, 0.0, keep["dx"][:, Dc:],
                             Dc + Dn, Dn, V, G)

    em = batch.event_mask.cpu()
    idx = batch.dynamic_indices.cpu()
    nnz = float((em.unsqueeze(-1) & (idx > 0)).sum())
    M = idx.shape[2]
    fbytes = nnz * (Dc + Dn) * 4 + B * Lq * M * 21 + B * Lq * G * (Dc + Dn) * 4 + float(em.sum()) * 2 * Dc * 4
    bbytes = nnz * (Dc + Dn) * 4 * G + nnz * 12 * 2 + V * (Dc + Dn) * 4
    return fwd, bwd, fbytes, bbytes, keep


def _c5_embed_bf16_microbench(dev, V_big: int = 1 << 22):
    """SURVEY.md §8d embed-bag microbench with a bf16 table far larger than the 256 MiB Infinity Cache: the C5 batch
    shape (B = 128, L = 1024, M = 32, nnz ~ 2.0 M) with every non-padding index redrawn uniformly over V = 2^22 rows
    x D = 256 bf16 (a 2 GiB table; padding 0 kept): ~1.6 M distinct rows, ~0.8 GB touched per launch, so the gathers
    leave L2 and the Infinity Cache (a bijection of the batch's own ~10 k vocabulary rows touched only ~5 MB and
    measured L2 hits). JOINT layer with static SUM_ALL and the temporal encoding (esgpt_embed_joint_fwd_ex).
    Per-occurrence bytes: every gathered row counted, 2 B per element; `achieved_counter_GBs` beside it is the
    DRAM-side figure of the PMC pass."""
    import ctypes

    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import batch_view, err_word
    from eventstreamgpt_amd.synthetic import CONFIGS

    bc = CONFIGS["C5"]
    batch = bc.batch(0, batch_size=128, device=dev)
    g = torch.Generator(device=dev).manual_seed(11)
    big = torch.randint(1, V_big, batch.dynamic_indices.shape, device=dev, generator=g)
    batch.dynamic_indices = torch.where(batch.dynamic_indices > 0, big, 0)
    sbig = torch.randint(1, V_big, batch.static_indices.shape, device=dev, generator=g)
    batch.static_indices = torch.where(batch.static_indices > 0, sbig, 0)
    D = 256
    table = torch.randn(V_big, D, device=dev, generator=torch.Generator(device=dev).manual_seed(7)).bfloat16()
    div = torch.exp(torch.arange(0, D, 2, device=dev).float() * (-torch.log(torch.tensor(1e4)).item() / D))
    out = torch.empty(128, batch.event_mask.shape[1], D, device=dev)
    lib = L.load()
    bv = batch_view(batch)
    err = err_word(dev)
    # as the input-layer operator runs it: the event times once per subject (esgpt_event_times), then the bag kernel
    # reading them as absolute times (both launches timed)
    times = torch.empty(batch.event_mask.shape, device=dev)
    tv = batch_view(batch)
    tv.struct.time_abs = times.data_ptr()
    flags = L.EMB_STATIC | L.EMB_TIME | L.EMB_TIME_ABS

    def fwd():
        L.check(lib.esgpt_event_times(tv.ref, times.data_ptr(), L.stream()), "event_times")
        L.check(lib.esgpt_embed_joint_fwd_ex(tv.ref, None, table.data_ptr(), L.BF16, V_big, D, div.data_ptr(),
                                             div.data_ptr(), flags, 0.5, 0.5, out.data_ptr(), err.data_ptr(),
                                             L.stream()), "embed_bf16")

    em = batch.event_mask
    B, Lq, M = batch.dynamic_indices.shape
    nnz = float((em.unsqueeze(-1) & (batch.dynamic_indices > 0)).sum())
    S = batch.static_indices.shape[1]
    nbytes = nnz * D * 2 + B * Lq * M * 21 + B * Lq * D * 4 + float(em.sum()) * S * D * 2 + B * Lq * 5
    return fwd, nbytes, nnz, (table, out, batch, div, times)


def roofline_entries(model, cfg, batch, dev, p_attn: float, cfg_name: str, dtype=torch.bfloat16) -> list:
    """The kernels measured for this configuration, at its own shapes: (name, symbol, bound, algorithmic work per
    launch, launcher, extras). Each launcher issues exactly one launch set of the kernel."""
    from eventstreamgpt_amd import _lib as L

    lib = L.load()
    B, Lq = batch.event_mask.shape
    D, H, F = cfg.hidden_size, cfg.num_attention_heads, cfg.intermediate_size
    hd = D // H
    T_pairs = attention_flops_fwd(batch, cfg) / (4.0 * H * hd)
    ents, keep = [], []

    def add(name, symbol, bound, work, fn, extra=None, hold=None):
        ents.append({"kernel": name, "symbol": symbol, "bound": bound, "work": work, "fn": fn, "extra": extra or {}})
        keep.append(hold)

    drop = p_attn > 0
    layer = f"{cfg_name} layer: B={B} H={H} L={Lq} hd={hd}, dropout {p_attn}"
    f32 = dtype == torch.float32
    fa, ba, ka, _ = _attention_launchers(B, Lq, D, H, batch.event_mask, p_attn, dev, dtype)
    add("attn_fwd", _attn_symbol(lib, True, hd, Lq, Lq, 3 * D, D, drop, dtype, B * H), "mfma",
        4.0 * H * hd * T_pairs, fa, {"shape": layer + " (global)"}, ka)
    add("attn_bwd", _attn_symbol(lib, False, hd, Lq, Lq, 3 * D, D, drop, dtype), "mfma", 8.0 * H * hd * T_pairs, ba,
        {"shape": layer + " (global)"}, None)
    gf, gb, kg = _gemm_launchers(B * Lq, D, F, dev, dtype)
    # the tile GEMM's rule (gemm.hip): 128x128 tiles when K and N >= 512 and M >= 4096, else 64x64 for c_fc
    wide = D >= 512 and F >= 512 and B * Lq >= 4096
    add("gemm_fc_fwd", "gemm_kernel<true, true, ..., F32>" if f32 else
        ("gemm_kernel<true, true, 3, 2, 2>" if wide else "gemm_kernel<true, true, 3, 1, 1>"), "mfma",
        2.0 * B * Lq * D * F, gf,
        {"shape": f"{cfg_name} c_fc: [{B * Lq}, {D}] x [{F}, {D}]^T + bias, GELU epilogue"
                  + (", f32 operands (v_mfma_f32_32x32x2_f32)" if f32 else "")}, kg)
    add("gemm_fc_bwd", "gemm_bwd_pair_kernel" + ("<..., F32>" if f32 else ""), "mfma", 4.0 * B * Lq * D * F, gb,
        {"shape": f"{cfg_name} c_fc backward: dX [{B * Lq}, {D}] + dW [{F}, {D}] f32 + db, one launch"
                  + (", f32 operands" if f32 else "")}, None)
    emb = model.encoder.input_layer.data_embedding_layer
    ci = cfg.structured_event_processing_mode == "conditionally_independent"
    if hasattr(emb, "embed_layer"):
        tl = model.encoder.input_layer.time_embedding_layer

        def emb_fwd():
            with torch.no_grad():
                emb.embed(batch, time_layer=tl)

        add("embed_joint_fwd", "embed_joint_fwd_kernel<4, 1>", "hbm", embed_fwd_bytes(batch, cfg), emb_fwd,
            {"shape": f"{cfg_name}: JOINT, B={B} L={Lq} V={emb.embed_layer.weight.shape[0]} D={D} f32 table"})
        eb, keb = _embed_bwd_launcher(model, batch)
        add("embed_joint_bwd", "bag_block_sort/col_prefix/row_scan/scatter/reduce/combine/subject kernels "
            "(esgpt_embed_bag_bwd)", "hbm", embed_bwd_bytes(batch, cfg), eb, {"shape": f"{cfg_name}: JOINT"}, keb)
    else:
        sf, sb, sfb, sbb, ks = _split_embed_launchers(model, batch)
        add("embed_split_fwd", "embed_split_bags_kernel<4>", "hbm", sfb, sf,
            {"shape": f"{cfg_name}: SPLIT cat/num bags, G={emb.n_levels} buckets, B={B} L={Lq}"}, ks)
        add("embed_split_bwd", "esgpt_embed_bag_bwd x2 (categorical + numerical selectors)", "hbm", sbb, sb,
            {"shape": f"{cfg_name}: SPLIT, G={emb.n_levels}"}, None)
    if ci:
        lf, lbytes, kl = _loss_launcher(model, batch, dtype)
        ln = "f32" if f32 else "bf16"
        add("output_loss", f"count_kernel + event_stream_kernel<{ln}> + reduce_kernel (esgpt_output_loss)", "hbm",
            lbytes, lf, {"shape": f"{cfg_name}: {ln} logits [{B * Lq}, {kl['zc'].shape[1]}]"}, kl)
    else:
        nf, nbytes, kn = _na_loss_launcher(model, batch)
        add("na_output_loss", "count_kernel + event_stream_kernel<bf16> + reduce_kernel (esgpt_output_loss, levels)",
            "hbm", nbytes, nf, {"shape": f"{cfg_name}: bf16 level rows [{kn['zc'].shape[0]}, {kn['zc'].shape[1]}] + "
                                         f"TTE rows [{kn['zt'].shape[0]}, {kn['zt'].shape[1]}]"}, kn)
    if cfg_name in ("C2", "C5"):
        cf, cbytes, nnz5, kc = _c5_embed_bf16_microbench(dev)
        add("embed_c5_bf16_microbench", "event_times_kernel + embed_joint_fwd_kernel<4, 1, bf16>", "hbm", cbytes, cf,
            {"shape": f"C5 batch shape B=128, L=1024, M=32, nnz={int(nnz5)}, indices uniform over a bf16 table "
                      "V=2^22 x 256 (2 GiB, 8x the Infinity Cache); per-occurrence bytes"}, kc)
    # long-sequence attention: MFMA efficiency once the grid fills the chip
    Bl, Ll, Hl = 4, 4096, 8
    fl, bl, kll, _ = _attention_launchers(Bl, Ll, Hl * hd, Hl, torch.ones(Bl, Ll, dtype=torch.bool, device=dev), 0.0,
                                          dev, dtype)
    long_pairs = Bl * Ll * (Ll + 1) / 2
    add("attn_fwd_long", _attn_symbol(lib, True, hd, Ll, Ll, 3 * Hl * hd, Hl * hd, False, dtype, Bl * Hl), "mfma",
        4.0 * Hl * hd * long_pairs, fl, {"shape": f"B={Bl} H={Hl} L={Ll} hd={hd}, causal, no dropout"}, kll)
    add("attn_bwd_long", _attn_symbol(lib, False, hd, Ll, Ll, 3 * Hl * hd, Hl * hd, False, dtype), "mfma",
        8.0 * Hl * hd * long_pairs, bl, {"shape": f"B={Bl} H={Hl} L={Ll} hd={hd}, causal, no dropout"}, None)
    for Bd in (B, 8 * B):
        fd, dbytes, kd = _decode_launcher(Bd, H, hd, Lq, dev)
        add("attn_decode" if Bd == B else "attn_decode_b8x", f"attn_decode_kernel<float, {hd}>", "hbm", dbytes, fd,
            {"shape": f"decode: B={Bd} H={H} hd={hd}, 1 query over a {Lq}-event f32 KV cache"}, kd)
    return ents, keep


def pmc_file(cfg_name: str) -> str:
    return os.path.join(REPO, "profiles", f"pmc_traffic_{cfg_name}.json")


def pmc_pass(model, cfg, batch, dev, p_attn: float, cfg_name: str, out_json: str, reps: int = 3) -> None:
    """The launches a rocprofv3 --pmc pass attributes (tools/pmc_traffic.py --entries): per roofline entry, one
    seed-bank launch as a marker, then ``reps`` eager launch sets of the entry; the entry names go to out_json."""
    from eventstreamgpt_amd.kernels import _seed_counter, begin_dropout_step

    ents, keep = roofline_entries(model, cfg, batch, dev, p_attn, cfg_name)
    _seed_counter(dev)
    for e in ents:
        e["fn"]()  # warm (lazy allocations, plans) before the counted launches
    torch.cuda.synchronize()
    for e in ents:
        begin_dropout_step(dev)  # marker: seed_bank_kernel
        for _ in range(reps):
            e["fn"]()
    begin_dropout_step(dev)
    torch.cuda.synchronize()
    with open(out_json, "w") as f:
        json.dump({"config": cfg_name, "reps": reps, "entries": [e["kernel"] for e in ents]}, f)


def roofline_report(model, cfg, batch, dev, p_attn: float, peak_tf: float, opt_cfg=None,
                    dtype=torch.bfloat16, cfg_name: str = "C2") -> tuple[dict, list]:
    """(roofline, roofline_aux): algorithmic work per launch / graph-replayed launch time, per kernel, at this
    configuration's shapes; ``traffic`` = HBM bytes per launch set from this configuration's own PMC passes
    (profiles/pmc_traffic_<config>.json), null when that file has no entry for the kernel."""
    traffic = {}
    pmc = pmc_file(cfg_name + ("" if dtype == torch.bfloat16 else "_f32"))  # counters of the same kernels only
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("bytes_per_launch", {})
    ents, keep = roofline_entries(model, cfg, batch, dev, p_attn, cfg_name, dtype)
    out = []
    for e in ents:
        ms = graph_time_ms(e["fn"])
        work = e["work"]
        if e["bound"] == "mfma":
            ach, peak, unit, wk = work / (ms * 1e-3) / 1e12, peak_tf, "TFLOP/s", "algorithmic_flops_per_launch"
        else:
            ach, peak, unit, wk = work / (ms * 1e-3) / 1e9, PEAK_HBM_GBS, "GB/s", "algorithmic_bytes_per_launch"
        r = {"kernel": e["kernel"], "symbol": e["symbol"], "bound": e["bound"], "achieved": round(ach, 3),
             "peak": peak, "unit": unit, "frac": round(ach / peak, 5), "traffic": traffic.get(e["kernel"]),
             "avg_ms": round(ms, 5), wk: work, "timing": "HIP graph of 20 launches, events on the replaying stream"}
        if e["bound"] == "hbm" and r["traffic"]:
            r["achieved_counter_GBs"] = round(r["traffic"] / (ms * 1e-3) / 1e9, 1)  # DRAM-side bytes / time
            r["frac_counter"] = round(r["achieved_counter_GBs"] / PEAK_HBM_GBS, 5)
        if e["bound"] == "hbm" and r["frac"] > 1.0:
            r["note"] = ("per-occurrence bytes (SURVEY 8d) count every gathered row; repeated rows are served from "
                         "L2 / MALL, so this exceeds the HBM peak: frac_counter is the DRAM-side fraction")
        r.update(e["extra"])
        out.append(r)
    # `roofline` = the step's dominant kernel by device time: the grouped projection backward (gemm_bwd_pair_kernel)
    # over EVERY launch shape of one step (frac = the step average); its c_fc launch alone is frac_isolated
    dom = next(i for i, e in enumerate(out) if e["kernel"] == "gemm_fc_bwd")
    d = out[dom]
    d["dominant"] = "largest share of the step's device time (grouped projection backward)"
    if opt_cfg is not None:
        ins = gemm_bwd_in_step(model, opt_cfg, batch, dtype)
        d["frac_isolated"], d["achieved_isolated"], d["avg_ms_isolated"] = d["frac"], d["achieved"], d["avg_ms"]
        d["achieved"] = round(ins["achieved"], 3)
        d["frac"] = round(ins["achieved"] / peak_tf, 5)
        d["avg_ms"] = round(ins["ms_per_step"] / ins["launches_per_step"], 5)
        d["algorithmic_flops_per_launch"] = round(d["achieved"] * 1e12 * d["avg_ms"] * 1e-3, 1)
        d["in_step"] = ins
        d["shape"] = f"{cfg_name}: every projection backward of one step ({ins['launches_per_step']} launches, " \
                     f"{len(ins['shapes'])} shapes, FLOP-weighted); traffic = the c_fc launch's"
    return d, out[:dom] + out[dom + 1:]


def cpu_baseline(bc, seconds: float = 12.0) -> dict:
    """The f32 oracle (CPU port of the reference step: fwd + bwd + AdamW) on this host's cores, B=4 subjects."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import esgpt_oracle as O
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    threads = torch.get_num_threads()
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = (CIPPTForGenerativeSequenceModeling if cfg.structured_event_processing_mode == "conditionally_independent"
         else NAPPTForGenerativeSequenceModeling)(cfg)  # the parameter layout the oracle reads
    trainable = {k for k, p in m.named_parameters() if p.requires_grad}
    params = {k: v.detach().clone().requires_grad_(k in trainable) for k, v in m.state_dict().items()}
    state = {}
    Bs = 4
    batch = bc.batch(0, batch_size=Bs)
    n_ev = float(batch.event_mask.sum())
    t0 = time.perf_counter()
    steps = 0
    while True:
        out = O.model_losses(params, cfg, batch)
        grads = torch.autograd.grad(out["loss"], [v for v in params.values() if v.requires_grad])
        named = dict(zip([k for k, v in params.items() if v.requires_grad], grads))
        with torch.no_grad():
            O.adamw_step({k: v for k, v in params.items() if v.requires_grad}, named, state, 1e-3, 0.01)
        steps += 1
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": steps * n_ev / dt, "unit": "train events/sec", "cores": threads, "kind": "port",
            "sample": f"{bc.name}: oracle f32 fwd+bwd+AdamW, B={Bs} subjects (L={bc.seq_len}), {steps} steps "
                      f"in {dt:.1f}s, torch.set_num_threads={threads}"}


def _launch_ranks(n: int) -> int:
    """``--gpus N`` outside torchrun: run this script under ``torch.distributed.run`` with N local ranks (a child
    process, started before this process touches the GPU) and return its exit status."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-hbm-line", action="store_true", help="skip the HBM-resident side measurement")
    ap.add_argument("--fuse-opt", action="store_true", help="measurement hook: the optimizer step captured at the "
                    "end of the step's graph (TrainStep fuse_optimizer; measured neutral on C2, off by default)")
    ap.add_argument("--no-check-errors", action="store_true", help="measurement hook: TrainStep(check_errors=False) "
                    "(no per-step error-word hand-off to the host)")
    ap.add_argument("--err-copy", action="store_true", help="measurement hook: each step's error words copied to "
                    "pinned host memory by a D2H copy on the compute stream (round 5) instead of written by the "
                    "optimizer launch into mapped host memory")
    ap.add_argument("--loss-pack", action="store_true", help="measurement hook: the replayed step's loss copy "
                    "made by its own pack launch instead of riding in the optimizer's prepare launch")
    ap.add_argument("--row-tiles", action="store_true", help="measurement hook: the dependency-graph projections "
                    "skip the padded events' row blocks (esgpt_gemm_row_tiles; off by default, measured no gain)")
    ap.add_argument("--opt-graph", action="store_true", help="replay the optimizer step as its own graph "
                    "(TrainStep capture_optimizer; measured ~10 us slower per C2 step, off by default)")
    ap.add_argument("--opt-host-args", action="store_true", help="measurement hook: host-computed lr / bias "
                    "corrections (round 3's optimizer launch) instead of the device schedule")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--roofline-only", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the roofline launches (clean step profiles)")
    ap.add_argument("--pmc-pass", default=None, help="with --roofline-only: the marker-separated launch sequence a "
                    "rocprofv3 --pmc pass attributes; entry names written to this JSON file")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args.gpus))
    rank, world, local = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    bc = CONFIGS[args.config]
    # Reference defaults: dropout 0.1 on inputs, residuals and attention probabilities (config.py:517-519).
    cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
    torch.manual_seed(0)
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    Model = (CIPPTForGenerativeSequenceModeling if cfg.structured_event_processing_mode == "conditionally_independent"
             else NAPPTForGenerativeSequenceModeling)
    model = Model(cfg).to(dev)
    model.train()
    opt_cfg = OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=10, max_training_steps=10_000)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    use_graph = not args.no_graph
    if args.loss_pack:
        from eventstreamgpt_amd import train as _train

        _train.LOSS_IN_OPT = False
    if args.err_copy:
        from eventstreamgpt_amd import train as _train

        _train.HOST_ERROR_WORDS = False
    if args.row_tiles:
        from eventstreamgpt_amd import fused

        fused.ROW_TILES = True
    ts = TrainStep(model, opt_cfg, compute_dtype=dtype, use_graph=use_graph, capture_optimizer=args.opt_graph,
                   check_errors=not args.no_check_errors, fuse_optimizer=args.fuse_opt)
    if args.opt_host_args:
        ts.opt.host_args = True

    n_batches = 4
    if args.roofline_only:  # the launches the PMC passes profile (no training steps)
        if args.pmc_pass:
            pmc_pass(model, cfg, bc.batch(0, device=dev), dev, 0.1, args.config, args.pmc_pass)
            return
        roofline, aux = roofline_report(model, cfg, bc.batch(0, device=dev), dev, 0.1,
                                        PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS,
                                        dtype=dtype, cfg_name=args.config)
        print(json.dumps({"roofline": roofline, "roofline_aux": aux}))
        return
    # Pre-collated batches in pinned host memory, packed like the native collate's output (one buffer per batch):
    # each step's H2D is one copy, issued on a copy stream while the previous step runs (TrainStep.prefetch).
    host = []
    for i in range(n_batches):
        b = bc.batch(100 * rank + i)
        hb = PytorchBatch.empty_packed({k: (tuple(v.shape), v.dtype) for k, v in b.as_dict().items()},
                                       pin_memory=True)
        hb.copy_(b)
        host.append(hb)
    events = [float(b.event_mask.sum()) for b in host]

    def timed(batches, prefetch: bool, steps: int, warmup: int):
        """Wall time of ``steps`` steps after ``warmup`` (barrier + synchronize on both sides), the median of per-step
        HIP-event times, and the events of the timed steps. ``prefetch``: host batches, each step's H2D issued on the
        copy stream during the previous step (TrainStep.prefetch)."""
        n = len(batches)
        if prefetch:
            ts.prefetch(batches[0])
        for i in range(warmup):
            ts.step(batches[i % n])
            if prefetch:
                ts.prefetch(batches[(i + 1) % n])
        ts.check()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        t0 = time.perf_counter()
        marks[0].record()
        for i in range(steps):
            j = warmup + i
            ts.step(batches[j % n])
            if prefetch:
                ts.prefetch(batches[(j + 1) % n])
            marks[i + 1].record()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        ts.check()
        st = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(steps))
        med = st[len(st) // 2] if len(st) % 2 else 0.5 * (st[len(st) // 2 - 1] + st[len(st) // 2])
        ev = sum(events[(warmup + i) % n] for i in range(steps))
        if world > 1:
            t = torch.tensor([el, med], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, med = float(t[0]), float(t[1])
            e = torch.tensor([ev], device=dev, dtype=torch.float64)
            dist.all_reduce(e)
            ev = float(e.item())
        return el, med, ev

    # value ("including H2D of the pre-collated batch"): the batches start in pinned host memory and
    # every step's H2D is inside the timed region (issued on a copy stream during the previous step, waited on by the
    # step). The rate on batches already resident in HBM is measured beside it (value_hbm_resident, never value).
    elapsed, median_ms, local_events = timed(host, True, args.steps, args.warmup)
    value = local_events / elapsed
    hbm = None
    if not args.no_hbm_line:
        dev_batches = [hb.to(dev) for hb in host]
        torch.cuda.synchronize()
        el_h, med_h, ev_h = timed(dev_batches, False, args.steps, args.warmup)
        hbm = {"value": round(ev_h / el_h, 1), "ms_per_step": round(1e3 * el_h / args.steps, 4),
               "ms_per_step_median": round(med_h, 4), "steps": args.steps, "warmup": args.warmup,
               "inputs": "batches resident in HBM; the step's only input copy is the D2D into the graph's static batch"}

    # ---- roofline: graph-replayed launches of the hot kernels on the step's shapes ----
    peak_tf = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
    roofline, aux = ({}, [])
    if rank == 0 and not args.no_roofline:
        roofline, aux = roofline_report(model, cfg, host[0].to(dev), dev, 0.1, peak_tf, opt_cfg, dtype, args.config)

    result = {
        "metric": "train events/sec (node)",
        "value": round(value, 1),
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "ms_per_step_median": round(median_ms, 4),
        "events_per_s_at_median": round(local_events / args.steps / (median_ms * 1e-3), 1),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
        "data": "synthetic (EHR-shaped batches, random-init weights); batches start in pinned host memory, each "
                "step's H2D inside the timed region (value_hbm_resident: batches already in HBM)",
        "config": {"workload": f"{args.config}: {bc.name}", "model": "CIPPT" if "CI" in bc.name else "NAPPT",
                   "global_batch": bc.batch_size * world, "seq_len": bc.seq_len, "parallelism": f"dp{world}",
                   "events_per_step_per_gpu": round(sum(events) / n_batches, 1), "hip_graph": ts.use_graph,
                   "dropout": {"input": 0.1, "resid": 0.1, "attention": 0.1}},
        "value_hbm_resident": hbm,
        "roofline": roofline,
        "roofline_aux": aux,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(bc)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
