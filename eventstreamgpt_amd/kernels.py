"""Python face of the custom operators (``torch.ops.esgpt``, defined in csrc/torch_ops.cpp; fake kernels and
autograd formulas in ``ops.py``) plus the per-device state they share: the device error block, the split-K /
cross-workgroup ticket array and the dropout seed bank.

Every function here launches through ``torch.ops.esgpt.*`` on torch's current HIP stream; outputs and workspaces
are allocated by torch (the library allocates nothing). Nothing here falls back to a CPU / ATen implementation: a
missing library or a non-HIP tensor raises ``HipExtensionMissing``. ``BatchView`` (the ``esgpt_batch`` ctypes
descriptor) remains for the raw C-ABI binding used by the ABI tests and the benchmark's isolated launches.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib as L
from .data.types import PytorchBatch


# ----------------------------------------------------------------------------------------------------------------
# Optional per-launch timing (HIP events on the launching stream); used by bench.py's roofline measurement.
# ----------------------------------------------------------------------------------------------------------------
TIMING = {"enabled": False, "events": {}}


class _timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if TIMING["enabled"]:
            self.s = torch.cuda.Event(enable_timing=True)
            self.e = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *a):
        if TIMING["enabled"]:
            self.e.record()
            TIMING["events"].setdefault(self.name, []).append((self.s, self.e))


def timing_summary() -> dict:
    """{name: (n_launches, mean_ms)} of the recorded launches (synchronises)."""
    torch.cuda.synchronize()
    out = {}
    for k, v in TIMING["events"].items():
        ms = [s.elapsed_time(e) for s, e in v]
        out[k] = (len(ms), sum(ms) / max(1, len(ms)))
    return out


# ----------------------------------------------------------------------------------------------------------------
# Batch view + device error word
# ----------------------------------------------------------------------------------------------------------------
class BatchView:
    """Device-resident, kernel-ready view of a ``PytorchBatch`` (contiguous tensors of the ABI's dtypes)."""

    def __init__(self, batch: PytorchBatch):
        dev = batch.event_mask.device
        if dev.type != "cuda":
            raise L.HipExtensionMissing("eventstreamgpt_amd kernels need the batch on a HIP device (no CPU path).")

        def c(t, dt):
            return None if t is None else t.to(dtype=dt).contiguous()

        self.event_mask = c(batch.event_mask, torch.bool)
        self.time_delta = c(batch.time_delta, torch.float32)
        self.time = c(batch.time, torch.float32)
        self.dyn_idx = c(batch.dynamic_indices, torch.int64)
        self.dyn_meas = c(batch.dynamic_measurement_indices, torch.int64)
        self.dyn_vals = c(batch.dynamic_values, torch.float32)
        self.dyn_vmask = c(batch.dynamic_values_mask, torch.bool)
        self.st_idx = c(batch.static_indices, torch.int64)
        self.st_meas = c(batch.static_measurement_indices, torch.int64)
        B, Lq, M = self.dyn_idx.shape
        S = 0 if self.st_idx is None else self.st_idx.shape[1]
        self.B, self.L, self.M, self.S = B, Lq, M, S
        self.struct = L.EsgptBatch(
            L.ptr(self.dyn_idx), L.ptr(self.dyn_meas), L.ptr(self.dyn_vals), L.ptr(self.dyn_vmask),
            L.ptr(self.event_mask), L.ptr(self.time_delta), L.ptr(self.time), L.ptr(self.st_idx),
            L.ptr(self.st_meas), B, Lq, M, S,
        )
        self.ref = ctypes.byref(self.struct)


def batch_view(batch: PytorchBatch) -> BatchView:
    """Builds (and caches on the batch object) the kernel view. The cache is keyed on the tensor storages."""
    key = (batch.event_mask.data_ptr(), batch.dynamic_indices.data_ptr(),
           None if batch.time is None else batch.time.data_ptr())
    v = getattr(batch, "_esgpt_view", None)
    if v is None or v[0] != key:
        v = (key, BatchView(batch))
        object.__setattr__(batch, "_esgpt_view", v)
    return v[1]


_ERR: dict[int, torch.Tensor] = {}
_LAST_V: dict[int, int] = {}


def _dev_index(device: torch.device) -> int:
    return device.index if device.index is not None else torch.cuda.current_device()


def err_word(device: torch.device) -> torch.Tensor:
    """The device error block of the C ABI (16 bytes: int32 ESGPT_FLAG_* bits, pad, int64 max bad index), viewed as
    int64 [2]. Kernels OR flags into it; esgpt_adamw is a no-op while the flags are set."""
    if device.type != "cuda":  # fake / meta tracing of the operators
        return torch.empty(2, dtype=torch.int64, device=device)
    idx = _dev_index(device)
    w = _ERR.get(idx)
    if w is None:
        w = torch.zeros(2, dtype=torch.int64, device=torch.device("cuda", idx))
        _ERR[idx] = w
    return w


def note_vocab(device: torch.device, V: int) -> None:
    """Remembers the table size of the latest embedding launch (the ``n_total_embeddings`` of its message)."""
    _LAST_V[_dev_index(device)] = int(V)


def raise_for_error(code: int, max_index: int, n_total_embeddings: int | None = None, batch=None) -> None:
    """The reference's exception for an error block's flags, in the reference's check order:
    ``torch._assert(indices.max() < V, f"Invalid embedding! {indices.max()} >= {V}")``
    (data_embedding_layer.py:485-488), then the TTE checks of get_TTE_outputs (model_output.py:1360-1367):
    ``ValueError(f"NaNs in TTE_LL: {batch}")`` before ``ValueError(f"No observed time-to-event for >= 1 patient in
    batch: {batch}")``."""
    code &= 0xFFFFFFFF
    if not code:
        return
    tail = "" if batch is None else f": {batch}"
    if code & L.FLAG_BAD_INDEX:
        raise AssertionError(f"Invalid embedding! {torch.tensor(max_index)} >= {n_total_embeddings}")  # 0-dim: prints the value
    if code & L.FLAG_TTE_NAN:
        raise ValueError(f"NaNs in TTE_LL{tail}")
    if code & L.FLAG_TTE_NO_OBS:
        raise ValueError(f"No observed time-to-event for >= 1 patient in batch{tail}")
    if code & L.FLAG_BAD_LABEL:
        raise IndexError("Target out of bounds in classification / regression labels")
    if code & L.FLAG_PEER_RANK:
        raise RuntimeError("eventstreamgpt_amd: a device error on another data-parallel rank in this step (its "
                           "exception is raised there); this rank skipped the step's update with it")
    raise RuntimeError(f"eventstreamgpt_amd: unknown device error flags {code:#x}")


def check_errors(device: torch.device | None = None, n_total_embeddings: int | None = None, batch=None):
    """Reads (one host sync) and clears the device error block; raises the reference's exception for its flags —
    the latest step's own, or the pending ones of an earlier step held in the sticky word (esgpt_step_begin).
    ``n_total_embeddings`` defaults to the table size of the latest embedding launch on the device."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    w = err_word(device)
    code, mx = (int(x) for x in w.tolist())
    if code:
        w.zero_()
        if n_total_embeddings is None:
            n_total_embeddings = _LAST_V.get(_dev_index(device))
        raise_for_error((code | (code >> 32)) & 0xFFFFFFFF, mx, n_total_embeddings, batch)


_TICKETS: dict[tuple[int, int], torch.Tensor] = {}
TICKETS_LEN = 1 << 16


def tickets(device: torch.device, slot: int = 0) -> torch.Tensor:
    """Per-device int32 counters of the kernels' in-launch last-arriver reductions (split-K GEMM tiles, column
    sums). Zeroed once here; every launch leaves the counters it used at zero. The launches that use one array are
    stream-ordered: slot 0 = the step's stream, slot 1 = the weight-gradient stream (``weight_grad_overlap``)."""
    if device.type != "cuda":  # fake / meta tracing of the operators
        return torch.empty(TICKETS_LEN, dtype=torch.int32, device=device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _TICKETS.get((idx, slot))
    if t is None:
        t = torch.zeros(TICKETS_LEN, dtype=torch.int32, device=torch.device("cuda", idx))
        _TICKETS[(idx, slot)] = t
    return t


_OVERLAP: set[int] = set()  # device indices whose projection backwards put dW on the weight-gradient stream


def weight_grad_overlap_active(device: torch.device) -> bool:
    return bool(_OVERLAP) and device.type == "cuda" and (
        device.index if device.index is not None else torch.cuda.current_device()) in _OVERLAP


class weight_grad_overlap:
    """Context of one backward pass: every projection backward (``esgpt::linear_bwd``) launches its input gradient
    on the current stream and its weight / bias gradient on the device's weight-gradient stream, so the dW products
    run beside the following layers' kernels instead of on backward's critical path. On exit (and whenever
    ``join`` is called, e.g. before a DDP bucket reads gradients) the current stream waits for that stream. Usable
    under HIP-graph capture (the fork / join become graph edges)."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.device = device
        self.enabled = enabled and device.type == "cuda"
        self.idx = (device.index if device.index is not None else torch.cuda.current_device()) if self.enabled else -1

    def __enter__(self):
        if self.enabled:
            _OVERLAP.add(self.idx)
        return self

    def join(self):
        if self.enabled:
            join_weight_grads(self.device)

    def __exit__(self, *exc):
        if self.enabled:
            _OVERLAP.discard(self.idx)
            join_weight_grads(self.device)
        return False


def _lib_partials(N: int) -> int:
    """Rows of a residual_ln backward partial table (esgpt_residual_ln_partials, at least 1)."""
    return max(1, int(L.load(require_device=False).esgpt_residual_ln_partials(N)))


_DEFER: dict[int, list] = {}  # device index -> pending (partials, sums) of deferred LayerNorm column sums


def _dev_idx(device: torch.device) -> int:
    return device.index if device.index is not None else torch.cuda.current_device()


def colsum_deferral_active(device: torch.device) -> bool:
    return bool(_DEFER) and device.type == "cuda" and _dev_idx(device) in _DEFER


def defer_colsum(device: torch.device, part: torch.Tensor, sums: torch.Tensor) -> None:
    _DEFER[_dev_idx(device)].append((part, sums))


def flush_colsums(device: torch.device) -> None:
    """Sums every pending LayerNorm-backward partial table of ``device`` in ONE launch (esgpt::colsum_flush)."""
    if device.type != "cuda":
        return
    pend = _DEFER.get(_dev_idx(device))
    if pend:
        _ops().colsum_flush([p for p, _ in pend], [s for _, s in pend])
        pend.clear()


class deferred_colsums:
    """Context of one backward pass: the LayerNorm backwards (``esgpt::residual_ln``'s registered backward) write
    only their per-block partials and hand autograd gradient tensors that one ``esgpt::colsum_flush`` launch fills
    on exit (or at ``flush_colsums``, e.g. before a DDP bucket reads gradients) — one launch instead of one per
    LayerNorm. Only gradients that go straight to leaf parameters are deferred (AccumulateGrad takes them without
    reading; TrainStep's accumulate guard flushes before any accumulation). Usable under HIP-graph capture."""

    def __init__(self, device: torch.device, enabled: bool = True):
        self.device = device
        self.enabled = enabled and device.type == "cuda"

    def __enter__(self):
        if self.enabled:
            _DEFER.setdefault(_dev_idx(self.device), [])
        return self

    def __exit__(self, *exc):
        if self.enabled:
            try:
                flush_colsums(self.device)
            finally:
                _DEFER.pop(_dev_idx(self.device), None)
        return False


_DEST: dict[int, tuple] = {}  # device index -> (recorder, destination | None) of the running training pass


class grad_destinations:
    """Context of one training pass (forward + backward) under DDP: the backward formulas write weight / bias
    gradients straight into the exchange buffer instead of fresh tensors (AccumulateGrad then takes the buffer's
    view as ``param.grad`` without a copy). ``recorder`` (a GradBuckets) learns, from the forward, which parameters
    one kernel output covers (``note_grad_group``: the q|k|v rows of one projection, a LayerNorm's (w, b) column
    sums, the padded head weights), so that its next layout keeps them adjacent; ``dest`` (the same object, or None
    when this pass must not write into the buffer — gradient accumulation, no-sync passes) hands out those regions
    (``grad_region``), each parameter at most once per pass."""

    def __init__(self, device: torch.device, recorder, dest):
        self.device = device
        self.enabled = recorder is not None and device.type == "cuda"
        self.recorder, self.dest = recorder, dest

    def __enter__(self):
        if self.enabled:
            if self.dest is not None:
                self.dest.begin_pass()
            _DEST[_dev_idx(self.device)] = (self.recorder, self.dest)
        return self

    def __exit__(self, *exc):
        if self.enabled:
            _DEST.pop(_dev_idx(self.device), None)
        return False


def note_grad_group(tensors, pad: int = 0) -> None:
    """Forward side: ``tensors`` (leaf parameters, in the order of one kernel output's rows) followed by ``pad``
    scratch elements are produced by one gradient kernel."""
    if _DEST and tensors and tensors[0] is not None and tensors[0].is_cuda:
        ent = _DEST.get(_dev_idx(tensors[0].device))
        if ent is not None:
            ent[0].note_group(tensors, pad)


def grad_region(tensors, pad: int = 0):
    """Backward side: the exchange buffer's f32 region holding ``tensors``' gradients back to back (+ ``pad``
    elements), claimed for this pass — or None (no destination active, a layout without this group, or a parameter
    already claimed: a second contribution is accumulated by autograd as usual)."""
    if not _DEST or not tensors or tensors[0] is None or not tensors[0].is_cuda:
        return None
    ent = _DEST.get(_dev_idx(tensors[0].device))
    if ent is None or ent[1] is None:
        return None
    return ent[1].region(tensors, pad)


def join_weight_grads(device: torch.device) -> None:
    """The current stream waits for every weight-gradient launch queued so far on ``device``."""
    _ops().weight_grad_join(tickets(device, 1))


def buckets_struct(groups: list[list] | None):
    """``split_by_measurement_indices`` → ``esgpt_buckets`` (None for the un-bucketed layer)."""
    if groups is None:
        return None
    if len(groups) > 8:
        raise ValueError("eventstreamgpt_amd supports at most 8 dependency-graph levels")
    s = L.EsgptBuckets()
    s.G = len(groups)
    for g, group in enumerate(groups):
        cb = nb = 0
        for entry in group:
            if isinstance(entry, (tuple, list)):
                mi, mode = entry
            else:
                mi, mode = entry, "categorical_and_numerical"
            mode = str(mode)
            if not 0 <= mi < 64:
                raise ValueError("eventstreamgpt_amd supports measurement indices < 64 in dependency-graph buckets")
            if mode in ("categorical_and_numerical", "categorical_only"):
                cb |= 1 << mi
            if mode in ("categorical_and_numerical", "numerical_only"):
                nb |= 1 << mi
            if mode not in ("categorical_and_numerical", "categorical_only", "numerical_only"):
                raise ValueError(f"Invalid group mode: {mode}")
        s.cat_bits[g] = cb
        s.num_bits[g] = nb
    return s


def _s64(u: int) -> int:
    return u - (1 << 64) if u >= (1 << 63) else u


def buckets_list(bk) -> list[int]:
    """``esgpt_buckets`` → the operators' ``int[] buckets`` ([] = un-bucketed; else G, cat_bits x8, num_bits x8)."""
    if bk is None:
        return []
    return [int(bk.G)] + [_s64(int(b)) for b in bk.cat_bits] + [_s64(int(b)) for b in bk.num_bits]


def _bref(bk):
    return None if bk is None else ctypes.byref(bk)


def _ops():
    from . import ops

    return ops.load()


def batch_args(batch: PytorchBatch) -> tuple:
    """The nine batch tensors of every input-layer / loss operator, in schema order."""
    if batch.event_mask.device.type != "cuda":
        raise L.HipExtensionMissing("eventstreamgpt_amd kernels need the batch on a HIP device (no CPU path).")
    return (batch.event_mask, batch.time_delta, batch.time, batch.dynamic_indices, batch.dynamic_measurement_indices,
            batch.dynamic_values, batch.dynamic_values_mask, batch.static_indices, batch.static_measurement_indices)


# ----------------------------------------------------------------------------------------------------------------
# Embedding
# ----------------------------------------------------------------------------------------------------------------
@dataclass
class EmbedSpec:
    flags: int
    static_w: float
    dynamic_w: float
    groups: list  # buckets_list(...) ([] = un-bucketed)
    G: int


def joint_embed(table, batch: PytorchBatch, spec: EmbedSpec, sin_div, cos_div):
    """``esgpt::embed_joint``: the JOINT DataEmbeddingLayer (+ time encoding / NA cumsum / mask) → f32 [B, L, G, D];
    differentiable in ``table``."""
    args = batch_args(batch)
    note_vocab(table.device, table.shape[0])
    with _timed("embed_joint_fwd"):
        return _ops().embed_joint(table, *args, spec.groups, sin_div, cos_div, spec.flags, float(spec.static_w),
                                  float(spec.dynamic_w), spec.G, err_word(table.device))


def split_bags(cat_table, num_table, batch: PytorchBatch, spec: EmbedSpec, cat_scale, num_scale, static_scale):
    """``esgpt::embed_split_bags``: SPLIT mode pre-projection bags X [B*L*G, Dc+Dn] =
    [cat_scale*bag_c + static_scale*static_c, num_scale*bag_n]; differentiable in both tables."""
    args = batch_args(batch)
    note_vocab(cat_table.device, cat_table.shape[0])
    return _ops().embed_split_bags(cat_table, num_table, *args, spec.groups, spec.flags, float(cat_scale),
                                   float(num_scale), float(static_scale), spec.G, err_word(cat_table.device))


def embed_epilogue(y, batch: PytorchBatch, G: int, flags: int, sin_div, cos_div):
    """``esgpt::embed_epilogue``: out[e,g] = mask_e * cumsum_g(y + time@g0) (flags select time / cumsum)."""
    return _ops().embed_epilogue(y, *batch_args(batch), G, flags, sin_div, cos_div)


class _SplitProjection(torch.autograd.Function):
    """SPLIT input projection + epilogue (data_embedding_layer.py:390-450 cat_proj / num_proj, then the temporal
    encoding / level cumsum / event mask): ``esgpt::split_proj_prep`` (the two weights column-concatenated in the
    GEMM dtype, the combined bias, the bags in the GEMM dtype — one launch), one GEMM with f32 output and the bias in
    its epilogue, ``esgpt::embed_epilogue``. Backward: the epilogue backward writes dy in the GEMM dtype, one grouped
    ``linear_bwd`` (dx, dW, db), ``esgpt::split_proj_post`` (dW column blocks and scaled bias gradients to the four
    parameters — straight into DDP exchange-buffer regions when active — and dx to f32). No framework kernels."""

    @staticmethod
    def forward(ctx, x, cat_w, num_w, cat_b, num_b, a_c, a_n, dt, batch, G, flags, sin_div, cos_div):
        ops = _ops()
        N, Dx = x.shape
        D, Dc = cat_w.shape
        x_lp, w_lp, bias = ops.split_proj_prep(x, cat_w, num_w, cat_b, num_b, float(a_c), float(a_n), dt)
        a = x_lp if dt == torch.bfloat16 else x
        y = torch.empty(N, D, dtype=torch.float32, device=x.device)
        ops.gemm_(y, L.GEMM_K_CONTIG, a, Dx, L.GEMM_K_CONTIG, w_lp, Dx, N, D, Dx, bias, None, False,
                  tickets(x.device))
        out = ops.embed_epilogue(y, *batch_args(batch), G, flags, sin_div, cos_div)
        ctx.save_for_backward(a, w_lp)
        ctx.batch, ctx.meta = batch, (G, flags, dt, Dc, float(a_c), float(a_n))
        ctx.params = (cat_w, num_w, cat_b, num_b)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .ops import _dest, _leaves, _linear_bwd

        a, w_lp = ctx.saved_tensors
        G, flags, dt, Dc, a_c, a_n = ctx.meta
        ops = _ops()
        dy = ops.embed_epilogue_bwd(dout.contiguous().float(), *batch_args(ctx.batch), G, flags, dt)
        need_dx = ctx.needs_input_grad[0]
        dx_lp, dw, db = _linear_bwd(dy, a, w_lp, None, -1, None, need_dx, True)
        ok = _leaves(*ctx.params)
        outs = []
        for p in ctx.params:
            r = _dest(ok, [p], 0, p.shape)
            outs.append(r if r is not None else torch.empty(p.shape, dtype=torch.float32, device=p.device))
        dx = ops.split_proj_post(dx_lp if (need_dx and dt == torch.bfloat16) else None, dw, db, Dc, a_c, a_n, *outs)
        if dt != torch.bfloat16:
            dx = dx_lp
        return (dx if need_dx else None, *outs) + (None,) * 8


def split_projection(x, cat_proj, num_proj, a_c: float, a_n: float, batch: PytorchBatch, G: int, flags: int,
                     sin_div, cos_div, dt):
    """SPLIT projection of the bag matrix x [B*L*G, Dc+Dn] (f32) + epilogue → f32 [B, L, G, D] (_SplitProjection);
    the GEMM runs in ``dt`` (bf16, or f32 in the reference-precision mode)."""
    return _SplitProjection.apply(x, cat_proj.weight, num_proj.weight, cat_proj.bias, num_proj.bias, a_c, a_n, dt,
                                  batch, G, flags, sin_div, cos_div)


def bag_bwd(batch: PytorchBatch, groups: list, selector: int, flags: int, dyn_scale: float, static_scale: float,
            dsrc, ld: int, D: int, V: int, G: int):
    """``esgpt::embed_bag_bwd``: the table gradient of the bag sums (dsrc rows of leading dimension ``ld``)."""
    return _ops().embed_bag_bwd(dsrc, *batch_args(batch), groups, selector, flags, float(dyn_scale),
                                float(static_scale), ld, D, V, G)


# ----------------------------------------------------------------------------------------------------------------
# Attention
# ----------------------------------------------------------------------------------------------------------------
_SEEDS: dict[int, torch.Tensor] = {}
_BANKS: dict[int, dict] = {}
SEED_BANK_SLOTS = 256


def _seed_counter(device: torch.device) -> torch.Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    c = _SEEDS.get(idx)
    if c is None:
        c = torch.full((1,), (torch.initial_seed() * 0x2545F491) & 0x7FFFFFFFFFFF, dtype=torch.int64, device=device)
        _SEEDS[idx] = c
    return c


def begin_dropout_step(device: torch.device, reset_errors: bool = False) -> None:
    """Refreshes the per-step seed bank on the stream (one small kernel per training step): slot i of the bank
    = counter + i, then counter += slots. Until the next call, ``next_dropout_seed`` hands out slots of the bank
    (no kernel per dropout site); under HIP-graph capture the refresh is part of the graph, so every replay draws
    fresh masks. Without a bank (eager use outside a step) every call clones and advances the counter.
    ``reset_errors``: the same launch zeroes the device error block (a training step's flags are its own)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    c = _seed_counter(device)
    bank = _BANKS.get(idx)
    if bank is None:
        bank = {"buf": torch.empty(SEED_BANK_SLOTS, dtype=torch.int64, device=device), "next": 0}
        _BANKS[idx] = bank
    _ops().seed_bank(c, bank["buf"], err_word(device) if reset_errors else None)  # one launch
    bank["next"] = 0


def next_dropout_seed(device: torch.device) -> torch.Tensor:
    """Device-side dropout seed (a 1-element int64 tensor that stays valid for the backward pass)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    bank = _BANKS.get(idx)
    if bank is not None and bank["next"] < SEED_BANK_SLOTS:
        i = bank["next"]
        bank["next"] = i + 1
        return bank["buf"][i: i + 1]
    c = _seed_counter(device)
    snap = c.clone()
    c.add_(1)
    return snap


def end_dropout_step(device: torch.device) -> None:
    """Closes the bank (later calls fall back to per-call seeds until the next ``begin_dropout_step``)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    bank = _BANKS.get(idx)
    if bank is not None:
        bank["next"] = SEED_BANK_SLOTS


def _attn_counters(device, B: int, H: int, Lk: int):
    """Exchange tickets of the attention backward's query-split workgroup pairs (None: unsplit launch)."""
    t = tickets(device)
    return t.data_ptr() if L.load().esgpt_attn_bwd_counters(B, H, Lk) <= t.numel() else None


def attention(qkv, key_mask, query_mask, H: int, window: int, static_kv_first: bool, dropout_p: float = 0.0):
    """``esgpt::attention``: packed-QKV causal / local attention. qkv: [Bs, T, 3D] (q | k | v), returns
    o: [Bs, T - skf, D]; differentiable in ``qkv`` (one fused MFMA backward)."""
    if qkv.device.type != "cuda":
        raise L.HipExtensionMissing("eventstreamgpt_amd: attention needs a HIP device tensor (no CPU path)")
    seed = next_dropout_seed(qkv.device) if dropout_p > 0 else None
    with _timed("attn_fwd"):
        o, _lse, _keep = _ops().attention(qkv, key_mask, query_mask, H, window, bool(static_kv_first), float(dropout_p),
                                   seed)
    return o


class AttentionFn:
    """Call-compatible name of ``attention`` (``AttentionFn.apply(qkv, key_mask, query_mask, H, window, skf, p)``)."""

    apply = staticmethod(attention)


# ----------------------------------------------------------------------------------------------------------------
# Generation: KV cache (csrc/decode.hip)
# ----------------------------------------------------------------------------------------------------------------
class _KVStore:
    """One layer's preallocated token-major cache, k / v: [B, cap, D]. ``length`` = rows written so far."""

    __slots__ = ("k", "v", "length", "H")

    def __init__(self, B: int, cap: int, D: int, H: int, dtype, device):
        self.k = torch.empty(B, cap, D, dtype=dtype, device=device)
        self.v = torch.empty(B, cap, D, dtype=dtype, device=device)
        self.length = 0
        self.H = H


class LayerKV(tuple):
    """``present_key_value`` of one layer: the reference's ``(key, value)`` pair, each [B, H, L, hd]
    (transformer.py:267), as views of a preallocated cache that the next decode step appends into in place
    (instead of the reference's per-step ``torch.cat``). A plain ``(key, value)`` tuple is accepted as a past too;
    it is copied into a fresh cache once."""

    def __new__(cls, store: _KVStore, length: int):
        B, _, D = store.k.shape
        H = store.H
        hd = D // H
        k = store.k[:, :length].view(B, length, H, hd).permute(0, 2, 1, 3)
        v = store.v[:, :length].view(B, length, H, hd).permute(0, 2, 1, 3)
        self = super().__new__(cls, (k, v))
        self.store = store
        self.length = length
        return self


def _kv_store_for(layer_past, B: int, D: int, H: int, n_new: int, cap_hint: int, dtype, device):
    """(store, past_len) with room for ``n_new`` more rows. Appends in place when ``layer_past`` is the newest view
    of its store (the usual decode loop); otherwise (a branched / foreign / full past) copies into a new store."""
    if isinstance(layer_past, LayerKV):
        st = layer_past.store
        P = layer_past.length
        if (st.length == P and P + n_new <= st.k.shape[1] and st.k.dtype == dtype and st.k.shape[0] == B
                and st.H == H and st.k.device == device):
            return st, P
    P = 0 if layer_past is None else int(layer_past[0].shape[-2])
    st = _KVStore(B, max(int(cap_hint), P + n_new), D, H, dtype, device)
    if P:
        pk, pv = layer_past[0], layer_past[1]
        if pk.shape[0] != B or pk.shape[1] * pk.shape[3] != D:
            raise ValueError(f"layer_past of shape {tuple(pk.shape)} does not match batch {B} / hidden size {D}")
        st.k[:, :P].copy_(pk.permute(0, 2, 1, 3).reshape(B, P, D))
        st.v[:, :P].copy_(pv.permute(0, 2, 1, 3).reshape(B, P, D))
    st.length = P
    return st, P


def cached_attention(qkv: torch.Tensor, layer_past, key_mask: torch.Tensor | None, H: int, window: int,
                     cap_hint: int):
    """Attention of the Lq new positions of packed ``qkv`` [B, Lq, 3D] over (past + new) keys, appending the new
    keys / values to the cache. ``key_mask``: bool [B, past + Lq] (the full event mask) or None. Returns
    (o [B, Lq, D], LayerKV). Inference only (no autograd through the cache)."""
    if torch.is_grad_enabled() and qkv.requires_grad:
        raise NotImplementedError("eventstreamgpt_amd: the KV-cache path is for generation (run under torch.no_grad())")
    if qkv.device.type != "cuda":
        raise L.HipExtensionMissing("eventstreamgpt_amd: KV-cache attention needs a HIP device tensor")
    ops = _ops()
    qkv = qkv.contiguous()
    B, Lq, D3 = qkv.shape
    D = D3 // 3
    hd = D // H
    st, P = _kv_store_for(layer_past, B, D, H, Lq, cap_hint, qkv.dtype, qkv.device)
    Lk = P + Lq
    cap = st.k.shape[1]
    with _timed("kv_append"):
        ops.kv_append(qkv, st.k, st.v, P)
    st.length = Lk
    km = qm = None
    if key_mask is not None:
        if tuple(key_mask.shape) != (B, Lk):
            raise ValueError(f"key mask of shape {tuple(key_mask.shape)} does not cover {Lk} keys of {B} subjects")
        km = key_mask.to(torch.bool).contiguous()
        qm = km[:, P:].contiguous()
    with _timed("attn_decode"):
        o = ops.attn_decode(qkv, st.k, st.v, km, qm, H, Lk, int(window))
    return o, LayerKV(st, Lk)


# ----------------------------------------------------------------------------------------------------------------
# Output-layer losses
# ----------------------------------------------------------------------------------------------------------------
def terms_list(terms) -> list[int]:
    """``esgpt_loss_term`` structs → the operators' flat ``int[] terms`` (8 ints per term)."""
    out = []
    for t in terms:
        out += [t.kind, t.meas_idx, t.vocab_start, t.vocab_end, t.col, t.obs_col, t.level, 0]
    return out


def tte_lists(tte) -> tuple[list[int], list[float]]:
    return [int(tte.kind), int(tte.K), int(tte.col)], [float(tte.mean_log), float(tte.std_log)]


def output_loss(zc, zt, zc_bias, batch: PytorchBatch, terms, tte, shift: int, n_levels: int):
    """``esgpt::output_loss``: fused generative losses. Returns f32 [n_terms + 2] = per-term losses, -TTE_LL,
    total. Only the total (last element) carries gradient; the per-term entries are for logging. ``zt=None`` means
    the TTE parameters live in ``zc`` (CI: one fused head GEMM)."""
    ti, tf = tte_lists(tte)
    with _timed("output_loss"):
        losses, _, _, _ = _ops().output_loss(zc, zt, zc_bias, *batch_args(batch), n_levels, shift,
                                             terms_list(terms), ti, tf, err_word(zc.device))
    return losses
