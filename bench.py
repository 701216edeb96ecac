"""Headline benchmark: CI-PPT training throughput (train events/sec) — BASELINE.json ``metric`` on ``configs[1]``
(C2: CI-PPT, 6 layers, d=256, L=256, global attention, synthetic EHR-shaped batches, one MI355X per rank).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-graph] [--no-cpu-baseline]
                    [--roofline-only] [--no-roofline]

A step = H2D of the pre-collated batch (pinned host -> HBM, overlapped with the previous step on a
copy stream) + forward + backward + (RCCL gradient all-reduce, overlapped with backward) + AdamW + LR-schedule
step on B=32 subjects per GPU (weak scaling). ``--gpus N`` without torchrun's environment re-launches this script
under ``torch.distributed.run`` with N ranks (before any GPU call) and exits with its status. Rank 0 prints ONE
JSON line: ``value`` = events of all ranks / wall time of the K timed steps (max over ranks, barrier +
synchronize on both sides); ``ms_per_step_median`` = the median step time from HIP events between steps.

Also reported (rank 0):
* ``roofline``: the step's dominant kernel by device time, the grouped projection backward (dX + dW + db of one
  Linear in one launch, MFMA-bound, 4·T·D·F algorithmic FLOPs) on c_fc's shape, timed in isolation (its launch
  captured 20 times into a HIP graph, replayed between HIP events on the capturing stream), plus ``frac_in_step``:
  the same kernel over EVERY launch shape of one step (shapes recorded from a real step, each timed likewise,
  FLOP-weighted). ``traffic`` = HBM bytes per launch from the committed rocprofv3 PMC summary
  (profiles/pmc_traffic.json: FETCH_SIZE doubled per the gfx950 calibration + WRITE_SIZE), when present.
* ``roofline_aux``: the same measurement for the attention forward / backward (4·H·hd·T /
  8·H·hd·T, T = allowed (query, key) pairs of the batch), the c_fc forward, the JOINT input layer forward and its
  table-gradient backward (HBM bytes, §8d per-occurrence accounting), the fused output-loss kernels (HBM bytes),
  the §8d C5 embed-bag microbench (B=128, L=1024, nnz ~ 2.0 M), a long-sequence attention forward and the
  generation decode kernel.
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


PMC_FILE = os.path.join(REPO, "profiles", "pmc_traffic.json")


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


def _attention_launchers(B, Lq, D, H, em, p, dev):
    """esgpt_attn_fwd / esgpt_attn_bwd launches on preallocated packed-qkv buffers (the step's layout)."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import tickets

    lib = L.load()
    hd = D // H
    g = torch.Generator(device=dev).manual_seed(0)
    bufs = {"qkv": (0.5 * torch.randn(B, Lq, 3 * D, device=dev, generator=g)).bfloat16(),
            "o": torch.empty(B, Lq, D, device=dev, dtype=torch.bfloat16),
            "lse": torch.empty(B, H, Lq, device=dev),
            "do": torch.randn(B, Lq, D, device=dev, generator=g).bfloat16(),
            "seed": torch.tensor([12345], dtype=torch.int64, device=dev),
            "em": em.to(torch.bool).contiguous()}
    bufs["dqkv"] = torch.empty_like(bufs["qkv"])
    nbytes = lib.esgpt_attn_bwd_workspace(B, H, Lq, Lq, hd)
    bufs["ws"] = torch.empty(max(1, nbytes), dtype=torch.uint8, device=dev)
    base, dbase, m, es = bufs["qkv"].data_ptr(), bufs["dqkv"].data_ptr(), bufs["em"].data_ptr(), 2
    cnt = tickets(torch.device(dev))

    def fwd():
        L.check(lib.esgpt_attn_fwd(base, base + D * es, base + 2 * D * es, 3 * D, Lq, bufs["o"].data_ptr(), D,
                                   bufs["lse"].data_ptr(), m, m, B, H, Lq, Lq, hd, 0, p, bufs["seed"].data_ptr(),
                                   L.BF16, L.stream()), "attn_fwd")

    def bwd():
        L.check(lib.esgpt_attn_bwd(base, base + D * es, base + 2 * D * es, 3 * D, Lq, bufs["o"].data_ptr(), D,
                                   bufs["do"].data_ptr(), D, bufs["lse"].data_ptr(), m, m, dbase, dbase + D * es,
                                   dbase + 2 * D * es, 3 * D, B, H, Lq, Lq, hd, 0, p, bufs["seed"].data_ptr(),
                                   L.BF16, bufs["ws"].data_ptr(), nbytes, cnt.data_ptr(), L.stream()), "attn_bwd")

    fwd()
    return fwd, bwd, bufs, cnt


def _gemm_launchers(T, D, F, dev):
    """c_fc on the step's shapes: forward with the bias + GELU epilogue, and its grouped backward."""
    from eventstreamgpt_amd import _lib as L
    from eventstreamgpt_amd.kernels import tickets

    lib = L.load()
    g = torch.Generator(device=dev).manual_seed(1)
    bufs = {"x": torch.randn(T, D, device=dev, generator=g).bfloat16(),
            "w": (0.05 * torch.randn(F, D, device=dev, generator=g)).bfloat16(),
            "b": torch.zeros(F, device=dev), "pre": torch.empty(T, F, device=dev, dtype=torch.bfloat16),
            "y": torch.empty(T, F, device=dev, dtype=torch.bfloat16),
            "dy": torch.randn(T, F, device=dev, generator=g).bfloat16(),
            "dx": torch.empty(T, D, device=dev, dtype=torch.bfloat16),
            "dw": torch.empty(F, D, device=dev), "db": torch.empty(F, device=dev)}
    nb = lib.esgpt_linear_bwd_workspace(T, D, F, 1)
    bufs["ws"] = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
    cnt = tickets(torch.device(dev))
    P = {k: v.data_ptr() for k, v in bufs.items()}

    def fwd():
        L.check(lib.esgpt_linear_fwd(P["x"], D, P["w"], T, D, F, P["b"], 0, P["pre"], P["y"], F, L.stream()),
                "linear_fwd")

    def bwd():
        L.check(lib.esgpt_linear_bwd(P["dy"], F, P["x"], D, P["w"], T, D, F, None, -1, None, 0, P["dx"], D, P["dw"],
                                     P["db"], P["ws"], nb, cnt.data_ptr(), L.stream()), "linear_bwd")

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


def _loss_launcher(model, batch):
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
    zc = torch.randn(B * Lq, C, device=dev, generator=g).bfloat16()
    bias = torch.zeros(C, device=dev).bfloat16()
    dzc = torch.empty_like(zc)
    dbias = torch.empty(B, C, device=dev)
    losses = torch.empty(len(terms) + 2, device=dev)
    nb = lib.esgpt_output_loss_workspace(B, Lq, len(terms))
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)
    arr = (L.EsgptLossTerm * max(1, len(terms)))(*terms)
    err = err_word(dev)

    def fwd():
        L.check(lib.esgpt_output_loss(bv.ref, zc.data_ptr(), C, 1, 1, bias.data_ptr(), zc.data_ptr(), C, L.BF16, arr,
                                      len(terms), ctypes.byref(tte), dzc.data_ptr(), dzc.data_ptr(),
                                      dbias.data_ptr(), losses.data_ptr(), ws.data_ptr(), nb, err.data_ptr(),
                                      L.stream()), "output_loss")

    nbytes = B * Lq * C * 2 * 2 + B * Lq * M * 21 + B * Lq * 5 + B * C * 4
    return fwd, float(nbytes), {"zc": zc, "dzc": dzc, "ws": ws, "arr": arr, "tte": tte}


def _c5_embed_microbench(dev):
    """SURVEY.md §8d embed-bag microbench: C5 vocabulary (V = 10,210), B = 128 subjects, L = 1024, M = 32
    (nnz ~ 2.0 M), JOINT layer with static SUM_ALL and the temporal encoding, forward only."""
    from eventstreamgpt_amd.synthetic import CONFIGS
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C5"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).to(dev)
    batch = bc.batch(0, batch_size=128, device=dev)
    emb = m.encoder.input_layer.data_embedding_layer
    tl = m.encoder.input_layer.time_embedding_layer

    def fwd():
        with torch.no_grad():
            emb.embed(batch, time_layer=tl)

    nnz = float((batch.event_mask.unsqueeze(-1) & (batch.dynamic_indices > 0)).sum())
    return fwd, embed_fwd_bytes(batch, cfg), nnz, (m, batch)


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
        dy = torch.randn(T, dout, device=dev, generator=g).bfloat16()
        x = torch.randn(T, din, device=dev, generator=g).bfloat16()
        w = torch.randn(dout, din, device=dev, generator=g).bfloat16()
        pre = torch.randn(T, din, device=dev, generator=g).bfloat16() if act >= 0 else None
        dx = torch.empty(T, din, device=dev, dtype=torch.bfloat16) if need_dx else None
        dw = torch.empty(dout, din, device=dev)
        db = torch.empty(dout, device=dev) if need_db else None
        nb = lib.esgpt_linear_bwd_workspace(T, din, dout, int(need_dx))
        ws = torch.empty(max(1, nb), dtype=torch.uint8, device=dev)

        def fn(dy=dy, x=x, w=w, pre=pre, dx=dx, dw=dw, db=db, ws=ws, nb=nb, T=T, din=din, dout=dout, act=act):
            L.check(lib.esgpt_linear_bwd(dy.data_ptr(), dout, x.data_ptr(), din, w.data_ptr(), T, din, dout, None, act,
                                         L.ptr(pre), din if pre is not None else 0, L.ptr(dx),
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


def roofline_report(model, cfg, batch, dev, p_attn: float, peak_tf: float, opt_cfg=None,
                    dtype=torch.bfloat16) -> tuple[dict, list]:
    """(roofline, roofline_aux): algorithmic work per launch / graph-replayed launch time, per kernel."""
    traffic = {}
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            traffic = json.load(f).get("bytes_per_launch", {})
    B, Lq = batch.event_mask.shape
    D, H, F = cfg.hidden_size, cfg.num_attention_heads, cfg.intermediate_size
    hd = D // H
    T_pairs = attention_flops_fwd(batch, cfg) / (4.0 * H * hd)
    entries = []

    def add(name, kernel, bound, work, fn, extra=None):
        ms = graph_time_ms(fn)
        if bound == "mfma":
            ach, peak, unit, wk = work / (ms * 1e-3) / 1e12, peak_tf, "TFLOP/s", "algorithmic_flops_per_launch"
        else:
            ach, peak, unit, wk = work / (ms * 1e-3) / 1e9, PEAK_HBM_GBS, "GB/s", "algorithmic_bytes_per_launch"
        tkey = (extra or {}).pop("traffic_key", kernel)
        e = {"kernel": name, "symbol": kernel, "bound": bound, "achieved": round(ach, 3), "peak": peak,
             "unit": unit, "frac": round(ach / peak, 5), "traffic": traffic.get(tkey), "avg_ms": round(ms, 5),
             wk: work, "timing": "HIP graph of 20 launches, events on the replaying stream"}
        e.update(extra or {})
        entries.append(e)

    drop = "true" if p_attn > 0 else "false"
    fa, ba, _keep_a, _ = _attention_launchers(B, Lq, D, H, batch.event_mask, p_attn, dev)
    add("attn_fwd", f"attn_fwd_mfma_kernel<{hd}, {drop}>", "mfma", 4.0 * H * hd * T_pairs, fa,
        {"shape": f"C2 layer: B={B} H={H} L={Lq} hd={hd}, dropout {p_attn}"})
    add("attn_bwd", f"attn_bwd_kernel<{hd}, {drop}>", "mfma", 8.0 * H * hd * T_pairs, ba,
        {"shape": f"C2 layer: B={B} H={H} L={Lq} hd={hd}, dropout {p_attn}"})
    gf, gb, _keep_g = _gemm_launchers(B * Lq, D, F, dev)
    add("gemm_fc_fwd", "gemm_kernel<true, true, 3, 1, 1>", "mfma", 2.0 * B * Lq * D * F, gf,
        {"shape": f"c_fc: [{B * Lq}, {D}] x [{F}, {D}]^T + bias, GELU epilogue"})
    add("gemm_fc_bwd", "gemm_bwd_pair_kernel", "mfma", 4.0 * B * Lq * D * F, gb,
        {"shape": f"c_fc backward: dX [{B * Lq}, {D}] + dW [{F}, {D}] f32 + db, one launch"})
    emb = model.encoder.input_layer.data_embedding_layer
    tl = model.encoder.input_layer.time_embedding_layer

    def emb_fwd():
        with torch.no_grad():
            emb.embed(batch, time_layer=tl)

    # the JOINT input layer and the CI loss layout only (the NA configuration's SPLIT bags and per-level loss rows
    # are timed inside its step)
    ci = cfg.structured_event_processing_mode == "conditionally_independent"
    if hasattr(emb, "embed_layer"):
        add("embed_joint_fwd", "embed_joint_fwd_kernel<4, 1>", "hbm", embed_fwd_bytes(batch, cfg), emb_fwd)
        eb, _keep_eb = _embed_bwd_launcher(model, batch)
        add("embed_joint_bwd", "bag_block_sort/col_prefix/row_scan/scatter/reduce/combine/subject kernels "
            "(esgpt_embed_bag_bwd)", "hbm",
            embed_bwd_bytes(batch, cfg), eb, {"traffic_key": "embed_bag_bwd"})
    if ci:
        lf, lbytes, _keep_lf = _loss_launcher(model, batch)
        add("output_loss", "count + event + reduce kernels (esgpt_output_loss)", "hbm", lbytes, lf,
            {"traffic_key": "output_loss", "shape": f"bf16 logits [{B * Lq}, {_keep_lf['zc'].shape[1]}]"})
    cf, cbytes, nnz5, _keep_c5 = _c5_embed_microbench(dev)
    add("embed_c5_microbench", "embed_joint_fwd_kernel<4, 1>", "hbm", cbytes, cf,
        {"traffic_key": "embed_joint_fwd_kernel@c5",
         "shape": f"C5 vocab V=10210, B=128, L=1024, M=32, nnz={int(nnz5)}, f32 table (per-occurrence bytes)"})
    # long-sequence attention: the forward kernel's MFMA efficiency once the grid fills the chip
    Bl, Ll, Hl = 4, 4096, 8
    fl, _, _keep_l, _ = _attention_launchers(Bl, Ll, Hl * hd, Hl, torch.ones(Bl, Ll, dtype=torch.bool, device=dev),
                                             0.0, dev)
    add("attn_fwd_long", f"attn_fwd_mfma_kernel<{hd}, false>", "mfma", 4.0 * Hl * hd * Bl * Ll * (Ll + 1) / 2, fl,
        {"shape": f"B={Bl} H={Hl} L={Ll} hd={hd}, causal, no dropout"})
    # generation: one decode step of the C2 model over a full cache, and a larger batch
    for Bd in (B, 8 * B):
        fd, dbytes, _keep_d = _decode_launcher(Bd, H, hd, Lq, dev)
        add("attn_decode" if Bd == B else "attn_decode_b256", f"attn_decode_kernel<float, {hd}>", "hbm", dbytes, fd,
            {"shape": f"decode: B={Bd} H={H} hd={hd}, 1 query over a {Lq}-event f32 KV cache",
             "traffic_key": f"attn_decode_kernel<float, {hd}>@grid{Bd * H * 256}"})
    # `roofline` = the step's dominant kernel by device time: the grouped projection backward (gemm_bwd_pair_kernel,
    # ~35 % of the C2 step in profiles/r01_c2_step_kernel_stats.csv), measured on c_fc's shape (its largest launch)
    dom = next(i for i, e in enumerate(entries) if e["kernel"] == "gemm_fc_bwd")
    entries[dom]["dominant"] = "largest share of the step's device time (grouped projection backward)"
    if opt_cfg is not None:
        ins = gemm_bwd_in_step(model, opt_cfg, batch, dtype)
        entries[dom]["frac_isolated"] = entries[dom]["frac"]
        entries[dom]["achieved_in_step"] = round(ins["achieved"], 3)
        entries[dom]["frac_in_step"] = round(ins["achieved"] / peak_tf, 5)
        entries[dom]["in_step"] = ins
    return entries[dom], entries[:dom] + entries[dom + 1:]


def cpu_baseline(bc, seconds: float = 12.0) -> dict:
    """The f32 oracle (CPU port of the reference step: fwd + bwd + AdamW) on this host's cores, B=4 subjects."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import esgpt_oracle as O
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    threads = torch.get_num_threads()
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg)
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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--roofline-only", action="store_true")
    ap.add_argument("--no-roofline", action="store_true", help="skip the roofline launches (clean step profiles)")
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
    ts = TrainStep(model, opt_cfg, compute_dtype=dtype, use_graph=use_graph)

    n_batches = 4
    if args.roofline_only:  # the launches the PMC passes profile (no training steps)
        roofline, aux = roofline_report(model, cfg, bc.batch(0, device=dev), dev, 0.1, PEAK_BF16_TFLOPS)
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

    ts.prefetch(host[0])
    for i in range(args.warmup):
        ts.step(host[i % n_batches])
        ts.prefetch(host[(i + 1) % n_batches])
    ts.check()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.steps):
        j = args.warmup + i
        ts.step(host[j % n_batches])
        ts.prefetch(host[(j + 1) % n_batches])
        marks[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ts.check()
    step_ms = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1]
                                                                            + step_ms[len(step_ms) // 2])
    local_events = sum(events[(args.warmup + i) % n_batches] for i in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed, median_ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, median_ms = float(t[0]), float(t[1])
        e = torch.tensor([local_events], device=dev, dtype=torch.float64)
        dist.all_reduce(e)
        local_events = float(e.item())
    value = local_events / elapsed

    # ---- roofline: graph-replayed launches of the hot kernels on the step's shapes ----
    peak_tf = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_F32_TFLOPS
    roofline, aux = ({}, [])
    if rank == 0 and not args.no_roofline:
        roofline, aux = roofline_report(model, cfg, host[0].to(dev), dev, 0.1, peak_tf, opt_cfg, dtype)

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
        "data": "synthetic (EHR-shaped batches, random-init weights); batches start in pinned host memory, the H2D "
                "copy is inside every timed step",
        "config": {"workload": f"{args.config}: {bc.name}", "model": "CIPPT" if "CI" in bc.name else "NAPPT",
                   "global_batch": bc.batch_size * world, "seq_len": bc.seq_len, "parallelism": f"dp{world}",
                   "events_per_step_per_gpu": round(sum(events) / n_batches, 1), "hip_graph": ts.use_graph,
                   "dropout": {"input": 0.1, "resid": 0.1, "attention": 0.1}},
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
