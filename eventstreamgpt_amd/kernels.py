"""Autograd wrappers around the C ABI (the PyTorch-ROCm custom-op layer).

Each ``torch.autograd.Function`` launches the gfx950 kernels on torch's current HIP stream with raw device
pointers; outputs and workspaces are allocated by torch (the library allocates nothing). Nothing here falls back
to a CPU / ATen implementation: a missing library or a non-CUDA tensor raises.
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
        raise AssertionError(f"Invalid embedding! {torch.tensor(max_index)} >= {n_total_embeddings}")
    if code & L.FLAG_TTE_NAN:
        raise ValueError(f"NaNs in TTE_LL{tail}")
    if code & L.FLAG_TTE_NO_OBS:
        raise ValueError(f"No observed time-to-event for >= 1 patient in batch{tail}")
    if code & L.FLAG_BAD_LABEL:
        raise IndexError("Target out of bounds in classification / regression labels")
    raise RuntimeError(f"eventstreamgpt_amd: unknown device error flags {code:#x}")


def check_errors(device: torch.device | None = None, n_total_embeddings: int | None = None, batch=None):
    """Reads (one host sync) and clears the device error block; raises the reference's exception for it.
    ``n_total_embeddings`` defaults to the table size of the latest embedding launch on the device."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    w = err_word(device)
    code, mx = (int(x) for x in w.tolist())
    if code:
        w.zero_()
        if n_total_embeddings is None:
            n_total_embeddings = _LAST_V.get(_dev_index(device))
        raise_for_error(code, mx, n_total_embeddings, batch)


_TICKETS: dict[int, torch.Tensor] = {}
TICKETS_LEN = 1 << 16


def tickets(device: torch.device) -> torch.Tensor:
    """Per-device int32 counters of the kernels' in-launch last-arriver reductions (split-K GEMM tiles, column
    sums). Zeroed once here; every launch leaves the counters it used at zero. The launches that use them are
    stream-ordered (one stream per device in the training step)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _TICKETS.get(idx)
    if t is None:
        t = torch.zeros(TICKETS_LEN, dtype=torch.int32, device=torch.device("cuda", idx))
        _TICKETS[idx] = t
    return t


def check_errors(device: torch.device | None = None, n_total_embeddings: int | None = None):
    """Reads (one host sync) and clears the device error word; raises the reference's exception for it."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    w = err_word(device)
    code = int(w.item())
    if code:
        w.zero_()
        if code & L.FLAG_BAD_INDEX:
            raise AssertionError(f"Invalid embedding! index >= {n_total_embeddings}")
        if code & L.FLAG_TTE_NO_OBS:
            raise ValueError("No observed time-to-event for >= 1 patient in batch")
        if code & L.FLAG_TTE_NAN:
            raise ValueError("NaNs in TTE_LL")
        if code & L.FLAG_BAD_LABEL:
            raise IndexError("Target out of bounds in classification / regression labels")


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


def _bref(bk):
    return None if bk is None else ctypes.byref(bk)


# ----------------------------------------------------------------------------------------------------------------
# Embedding
# ----------------------------------------------------------------------------------------------------------------
@dataclass
class EmbedSpec:
    flags: int
    static_w: float
    dynamic_w: float
    groups: object  # EsgptBuckets or None
    G: int


def _bag_bwd(bv, spec_groups, selector, flags, dyn_scale, static_scale, dsrc, ld, D, V, G):
    lib = L.load()
    dtable = torch.empty(V, D, dtype=torch.float32, device=dsrc.device)
    nbytes = lib.esgpt_embed_bag_bwd_workspace(bv.ref, G, V, D)
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=dsrc.device)
    L.check(lib.esgpt_embed_bag_bwd(bv.ref, _bref(spec_groups), selector, flags, dyn_scale, static_scale,
                                    dsrc.data_ptr(), ld, D, V, dtable.data_ptr(), ws.data_ptr(), nbytes, L.stream()),
            "embed_bag_bwd")
    return dtable


def _epilogue_bwd(bv, G, D, dout, flags):
    lib = L.load()
    dy = torch.empty_like(dout)
    L.check(lib.esgpt_embed_epilogue_bwd(bv.ref, G, D, dout.data_ptr(), flags, dy.data_ptr(), L.stream()),
            "embed_epilogue_bwd")
    return dy


class JointEmbedFn(torch.autograd.Function):
    """JOINT DataEmbeddingLayer (+ optional time encoding / NA cumsum) → f32 [B, L, G, D]."""

    @staticmethod
    def forward(ctx, table, bv: BatchView, spec: EmbedSpec, sin_div, cos_div):
        lib = L.load()
        V, D = table.shape
        table = table.contiguous().float()
        out = torch.empty(bv.B, bv.L, spec.G, D, dtype=torch.float32, device=table.device)
        note_vocab(table.device, V)
        with _timed("embed_joint_fwd"):
            st = lib.esgpt_embed_joint_fwd(bv.ref, _bref(spec.groups), table.data_ptr(), V, D, L.ptr(sin_div),
                                           L.ptr(cos_div), spec.flags, spec.static_w, spec.dynamic_w,
                                           out.data_ptr(), err_word(table.device).data_ptr(), L.stream())
        L.check(st, "embed_joint_fwd")
        ctx.bv, ctx.spec, ctx.V, ctx.D = bv, spec, V, D
        return out

    @staticmethod
    def backward(ctx, dout):
        bv, spec, V, D = ctx.bv, ctx.spec, ctx.V, ctx.D
        dout = dout.contiguous().float()
        if spec.flags & L.EMB_CUMSUM:
            dsrc = _epilogue_bwd(bv, spec.G, D, dout, spec.flags)
        else:
            dsrc = dout
        static = bool(spec.flags & L.EMB_STATIC) and bv.S > 0
        dyn_scale = spec.dynamic_w if static else 1.0
        with _timed("embed_joint_bwd"):
            dtable = _bag_bwd(bv, spec.groups, L.BAG_JOINT, spec.flags, dyn_scale, spec.static_w, dsrc, D, D, V,
                              spec.G)
        return dtable, None, None, None, None


class SplitBagsFn(torch.autograd.Function):
    """SPLIT mode pre-projection bags: X [B*L*G, Dc+Dn] = [cat_scale*bag_c + static_scale*static_c, num_scale*bag_n]."""

    @staticmethod
    def forward(ctx, cat_table, num_table, bv: BatchView, spec: EmbedSpec, cat_scale, num_scale, static_scale):
        lib = L.load()
        V, Dc = cat_table.shape
        Dn = num_table.shape[1]
        cat_table = cat_table.contiguous().float()
        num_table = num_table.contiguous().float()
        x = torch.empty(bv.B * bv.L * spec.G, Dc + Dn, dtype=torch.float32, device=cat_table.device)
        note_vocab(cat_table.device, V)
        L.check(lib.esgpt_embed_split_bags_fwd(bv.ref, _bref(spec.groups), cat_table.data_ptr(), Dc,
                                               num_table.data_ptr(), Dn, V, spec.flags, cat_scale, num_scale,
                                               static_scale, x.data_ptr(), err_word(x.device).data_ptr(),
                                               L.stream()), "embed_split_bags_fwd")
        ctx.bv, ctx.spec, ctx.V, ctx.Dc, ctx.Dn = bv, spec, V, Dc, Dn
        ctx.scales = (cat_scale, num_scale, static_scale)
        return x

    @staticmethod
    def backward(ctx, dx):
        bv, spec, V, Dc, Dn = ctx.bv, ctx.spec, ctx.V, ctx.Dc, ctx.Dn
        cat_scale, num_scale, static_scale = ctx.scales
        dx = dx.contiguous().float()
        flags = spec.flags
        if static_scale == 0.0:
            flags &= ~L.EMB_STATIC
        dcat = _bag_bwd(bv, spec.groups, L.BAG_CAT, flags, cat_scale, static_scale, dx, Dc + Dn, Dc, V, spec.G)
        dnum = _bag_bwd(bv, spec.groups, L.BAG_NUM, flags, num_scale, 0.0, dx[:, Dc:], Dc + Dn, Dn, V, spec.G)
        return dcat, dnum, None, None, None, None, None


class EmbedEpilogueFn(torch.autograd.Function):
    """out[e,g] = mask_e * cumsum_g(y + time@g0) (flags select time / cumsum)."""

    @staticmethod
    def forward(ctx, y, bv: BatchView, G, flags, sin_div, cos_div):
        lib = L.load()
        D = y.shape[-1]
        y = y.contiguous().float()
        out = torch.empty(bv.B, bv.L, G, D, dtype=torch.float32, device=y.device)
        L.check(lib.esgpt_embed_epilogue_fwd(bv.ref, G, D, y.data_ptr(), L.ptr(sin_div), L.ptr(cos_div), flags,
                                             out.data_ptr(), L.stream()), "embed_epilogue_fwd")
        ctx.bv, ctx.G, ctx.D, ctx.flags = bv, G, D, flags
        return out

    @staticmethod
    def backward(ctx, dout):
        dy = _epilogue_bwd(ctx.bv, ctx.G, ctx.D, dout.contiguous().float(), ctx.flags)
        return dy.view(-1, ctx.D), None, None, None, None, None


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


def begin_dropout_step(device: torch.device) -> None:
    """Refreshes the per-step seed bank on the stream (two small kernels per training step): slot i of the bank
    = counter + i, then counter += slots. Until the next call, ``next_dropout_seed`` hands out slots of the bank
    (no kernel per dropout site); under HIP-graph capture the refresh is part of the graph, so every replay draws
    fresh masks. Without a bank (eager use outside a step) every call clones and advances the counter."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    c = _seed_counter(device)
    bank = _BANKS.get(idx)
    if bank is None:
        bank = {"buf": torch.empty(SEED_BANK_SLOTS, dtype=torch.int64, device=device),
                "ar": torch.arange(SEED_BANK_SLOTS, dtype=torch.int64, device=device), "next": 0}
        _BANKS[idx] = bank
    torch.add(bank["ar"], c, out=bank["buf"])
    c.add_(SEED_BANK_SLOTS)
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


class AttentionFn(torch.autograd.Function):
    """Packed-QKV causal/local attention. qkv: [Bs, T, 3D] (q | k | v), returns o: [Bs, T - skf, D]."""

    @staticmethod
    def forward(ctx, qkv, key_mask, query_mask, H: int, window: int, static_kv_first: bool, dropout_p: float = 0.0):
        lib = L.load()
        qkv = qkv.contiguous()
        Bs, T, D3 = qkv.shape
        D = D3 // 3
        hd = D // H
        skf = 1 if static_kv_first else 0
        Lk, Lq = T, T - skf
        es = qkv.element_size()
        base = qkv.data_ptr()
        o = torch.empty(Bs, Lq, D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(Bs, H, Lq, dtype=torch.float32, device=qkv.device)
        seed = next_dropout_seed(qkv.device) if dropout_p > 0 else None
        with _timed("attn_fwd"):
            st = lib.esgpt_attn_fwd(base + skf * D3 * es, base + D * es, base + 2 * D * es, D3, T, o.data_ptr(), D,
                                    lse.data_ptr(), L.ptr(key_mask), L.ptr(query_mask), Bs, H, Lq, Lk, hd, window,
                                    float(dropout_p), L.ptr(seed), L.dtype_code(qkv.dtype), L.stream())
        L.check(st, "attn_fwd")
        ctx.save_for_backward(qkv, o, lse, key_mask, query_mask, seed)
        ctx.cfg = (H, window, skf, float(dropout_p))
        return o

    @staticmethod
    def backward(ctx, do):
        lib = L.load()
        qkv, o, lse, key_mask, query_mask, seed = ctx.saved_tensors
        H, window, skf, dropout_p = ctx.cfg
        do = do.contiguous().to(qkv.dtype)
        Bs, T, D3 = qkv.shape
        D = D3 // 3
        hd = D // H
        Lk, Lq = T, T - skf
        es = qkv.element_size()
        dqkv = (torch.zeros if skf else torch.empty)(Bs, T, D3, dtype=qkv.dtype, device=qkv.device)
        nbytes = lib.esgpt_attn_bwd_workspace(Bs, H, Lq, Lk, hd)
        ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=qkv.device)
        base, dbase = qkv.data_ptr(), dqkv.data_ptr()
        with _timed("attn_bwd"):
            st = lib.esgpt_attn_bwd(base + skf * D3 * es, base + D * es, base + 2 * D * es, D3, T, o.data_ptr(), D,
                                    do.data_ptr(), D, lse.data_ptr(), L.ptr(key_mask), L.ptr(query_mask),
                                    dbase + skf * D3 * es, dbase + D * es, dbase + 2 * D * es, D3, Bs, H, Lq, Lk, hd,
                                    window, dropout_p, L.ptr(seed), L.dtype_code(qkv.dtype), ws.data_ptr(), nbytes,
                                    _attn_counters(qkv.device, Bs, H, Lk), L.stream())
        L.check(st, "attn_bwd")
        return dqkv, None, None, None, None, None, None


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
    lib = L.load()
    if qkv.device.type != "cuda":
        raise L.HipExtensionMissing("eventstreamgpt_amd: KV-cache attention needs a HIP device tensor")
    qkv = qkv.contiguous()
    B, Lq, D3 = qkv.shape
    D = D3 // 3
    hd = D // H
    st, P = _kv_store_for(layer_past, B, D, H, Lq, cap_hint, qkv.dtype, qkv.device)
    Lk = P + Lq
    cap = st.k.shape[1]
    code = L.dtype_code(qkv.dtype)
    with _timed("kv_append"):
        s = lib.esgpt_kv_append(qkv.data_ptr(), D3, st.k.data_ptr(), st.v.data_ptr(), B, Lq, P, cap, D, code,
                                L.stream())
    L.check(s, "kv_append")
    st.length = Lk
    km = qm = None
    if key_mask is not None:
        if tuple(key_mask.shape) != (B, Lk):
            raise ValueError(f"key mask of shape {tuple(key_mask.shape)} does not cover {Lk} keys of {B} subjects")
        km = key_mask.to(torch.bool).contiguous()
        qm = km[:, P:].contiguous()
    o = torch.empty(B, Lq, D, dtype=qkv.dtype, device=qkv.device)
    with _timed("attn_decode"):
        s = lib.esgpt_attn_decode(qkv.data_ptr(), D3, st.k.data_ptr(), st.v.data_ptr(), L.ptr(km), L.ptr(qm),
                                  o.data_ptr(), D, B, H, Lq, Lk, cap, hd, int(window), code, L.stream())
    L.check(s, "attn_decode")
    return o, LayerKV(st, Lk)


# ----------------------------------------------------------------------------------------------------------------
# Output-layer losses
# ----------------------------------------------------------------------------------------------------------------
class OutputLossFn(torch.autograd.Function):
    """Fused generative losses. Returns f32 [n_terms + 2] = per-term losses, -TTE_LL, total.

    Only the total (last element) carries gradient; the per-term entries are for logging.
    ``zt=None`` means the TTE parameters live in ``zc`` (CI: one fused head GEMM).
    """

    @staticmethod
    def forward(ctx, zc, zt, zc_bias, bv: BatchView, terms, tte, shift: int, n_levels: int):
        lib = L.load()
        zc = zc.contiguous()
        ldc = zc.shape[-1]
        same = zt is None
        zt_ = zc if same else zt.contiguous()
        ldt = zt_.shape[-1]
        if zc_bias is not None:
            zc_bias = zc_bias.to(zc.dtype).contiguous()
        n_terms = len(terms)
        arr = (L.EsgptLossTerm * max(1, n_terms))(*terms)
        dzc = torch.empty_like(zc)
        dzt = dzc if same else torch.empty_like(zt_)
        dbias = torch.empty(bv.B, ldc, dtype=torch.float32, device=zc.device) if shift else None
        losses = torch.empty(n_terms + 2, dtype=torch.float32, device=zc.device)
        nbytes = lib.esgpt_output_loss_workspace(bv.B, bv.L, n_terms)
        ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=zc.device)
        with _timed("output_loss"):
            st = lib.esgpt_output_loss(bv.ref, zc.data_ptr(), ldc, n_levels, shift, L.ptr(zc_bias), zt_.data_ptr(),
                                       ldt, L.dtype_code(zc.dtype), arr, n_terms, ctypes.byref(tte), dzc.data_ptr(),
                                       dzt.data_ptr(), L.ptr(dbias), losses.data_ptr(), ws.data_ptr(), nbytes,
                                       err_word(zc.device).data_ptr(), L.stream())
        L.check(st, "output_loss")
        ctx.same = same
        ctx.has_bias = zc_bias is not None
        ctx.save_for_backward(dzc, None if same else dzt, dbias)
        return losses

    @staticmethod
    def backward(ctx, g):
        dzc, dzt, dbias = ctx.saved_tensors
        gt = g[-1].to(dzc.dtype)
        d_zc = dzc * gt
        d_zt = None if ctx.same else dzt * gt
        d_bias = (dbias.sum(0) * g[-1]) if (ctx.has_bias and dbias is not None) else None
        return d_zc, d_zt, d_bias, None, None, None, None, None
