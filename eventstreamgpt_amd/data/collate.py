"""Batch producer: ragged event streams -> a padded ``PytorchBatch`` through the native collate (``esgpt_collate``).

Mirrors ``PytorchDataset.collate`` (``EventStream/data/pytorch_dataset.py:527-701``). The reference pads one
event at a time in Python and tensorises through float32 (~per-event ``torch.Tensor`` + ``F.pad`` calls). Here a
batch is a set of windows into one flat store (``RaggedEvents``: the DL_reps columns as contiguous arrays plus
offsets), and the C++ collate writes every output field in one multithreaded pass into (optionally pinned)
host buffers, ready for one non-blocking copy to HBM.

Differences from the reference, all deliberate:
* indices are copied exactly as int64 (the reference's float32 round trip is exact only below 2**24);
* a ``None`` event index list is an empty event here (the reference raises ``TypeError`` on it in ``len``).
"""
from __future__ import annotations

import dataclasses
import os

import numpy as np
import torch

from .. import _lib
from .types import PytorchBatch

_NAN = float("nan")


@dataclasses.dataclass
class RaggedEvents:
    """Subjects as flat arrays. Subject s: events ``ev_start[s] .. ev_start[s] + ev_count[s] - 1``; event e:
    elements ``el_off[e] .. el_off[e+1] - 1``; static elements ``st_start[s] .. st_start[s] + st_count[s] - 1``.
    ``time_delta`` and ``vals`` are float64 with NaN for missing; ``idx`` / ``meas`` int64 (0 for missing)."""

    ev_start: np.ndarray
    ev_count: np.ndarray
    time_delta: np.ndarray
    el_off: np.ndarray
    idx: np.ndarray
    meas: np.ndarray
    vals: np.ndarray
    st_start: np.ndarray | None = None
    st_count: np.ndarray | None = None
    st_idx: np.ndarray | None = None
    st_meas: np.ndarray | None = None

    @property
    def n_subjects(self) -> int:
        return int(self.ev_start.shape[0])

    def __post_init__(self):
        i64 = lambda a: None if a is None else np.ascontiguousarray(a, dtype=np.int64)  # noqa: E731
        f64 = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731
        self.ev_start, self.ev_count, self.el_off = i64(self.ev_start), i64(self.ev_count), i64(self.el_off)
        self.idx, self.meas = i64(self.idx), i64(self.meas)
        self.time_delta, self.vals = f64(self.time_delta), f64(self.vals)
        self.st_start, self.st_count = i64(self.st_start), i64(self.st_count)
        self.st_idx, self.st_meas = i64(self.st_idx), i64(self.st_meas)
        n_ev = self.time_delta.shape[0]
        if self.el_off.shape[0] != n_ev + 1 or self.ev_start.shape != self.ev_count.shape:
            raise ValueError("RaggedEvents: el_off must hold n_events + 1 offsets; ev_start/ev_count must match")
        if (self.ev_start.size and (self.ev_start.min() < 0 or (self.ev_start + self.ev_count).max() > n_ev)):
            raise ValueError("RaggedEvents: a subject's events fall outside the event arrays")
        nnz = int(self.el_off[-1])
        if not (self.idx.shape[0] >= nnz and self.meas.shape[0] >= nnz and self.vals.shape[0] >= nnz):
            raise ValueError("RaggedEvents: element arrays shorter than el_off[-1]")
        if self.st_count is not None:
            ns = 0 if self.st_count.size == 0 else int((self.st_start + self.st_count).max())
            if self.st_idx.shape[0] < ns or self.st_meas.shape[0] < ns:
                raise ValueError("RaggedEvents: static arrays shorter than the static offsets")

    def window(self, subjects, starts=None, counts=None) -> "RaggedEvents":
        """A batch view: the given subjects, optionally restricted to ``counts`` events from ``starts`` (relative
        to each subject's first event). Shares every element array (no copy)."""
        subjects = np.asarray(subjects, dtype=np.int64)
        ev_start = self.ev_start[subjects].copy()
        ev_count = self.ev_count[subjects].copy()
        if starts is not None:
            starts = np.asarray(starts, dtype=np.int64)
            if (starts < 0).any() or (starts > ev_count).any():
                raise ValueError("window: start outside the subject's events")
            ev_start += starts
            ev_count -= starts
        if counts is not None:
            ev_count = np.minimum(ev_count, np.asarray(counts, dtype=np.int64))
        return RaggedEvents(
            ev_start, ev_count, self.time_delta, self.el_off, self.idx, self.meas, self.vals,
            None if self.st_start is None else self.st_start[subjects],
            None if self.st_count is None else self.st_count[subjects], self.st_idx, self.st_meas)


def _num(v):
    return _NAN if v is None else v


def flatten_items(items: list[dict], static: bool = True) -> RaggedEvents:
    """Reference ``__getitem__``-format dicts -> one ``RaggedEvents``. (The reader's own path never builds these
    dicts; this is the drop-in for callers that hand ``collate`` a list of items.)"""
    ev_count = np.array([len(e["time_delta"]) for e in items], dtype=np.int64)
    ev_start = np.concatenate([[0], np.cumsum(ev_count)[:-1]]) if len(items) else np.zeros(0, np.int64)
    td, lens, idx, meas, vals = [], [], [], [], []
    for e in items:
        td.extend(_num(t) for t in e["time_delta"])
        di, dm, dv = e["dynamic_indices"], e["dynamic_measurement_indices"], e["dynamic_values"]
        for j in range(len(e["time_delta"])):
            ii = di[j] or []
            n = len(ii)
            mm = (dm[j] or []) if dm is not None else []
            vv = (dv[j] or []) if dv is not None else []
            lens.append(n)
            idx.extend(0 if v is None else v for v in ii)
            meas.extend(0 if v is None else v for v in mm[:n])
            meas.extend([0] * (n - min(n, len(mm))))
            vals.extend(_num(v) for v in vv[:n])
            vals.extend([_NAN] * (n - min(n, len(vv))))
    el_off = np.concatenate([[0], np.cumsum(np.asarray(lens, dtype=np.int64))])
    st = {}
    if static:
        st_count = np.array([len(e["static_indices"]) for e in items], dtype=np.int64)
        st["st_count"] = st_count
        st["st_start"] = np.concatenate([[0], np.cumsum(st_count)[:-1]]) if len(items) else st_count
        st["st_idx"] = np.array([v for e in items for v in e["static_indices"]], dtype=np.int64)
        st["st_meas"] = np.array([v for e in items for v in e["static_measurement_indices"]], dtype=np.int64)
    return RaggedEvents(ev_start, ev_count, np.asarray(td, dtype=np.float64), el_off,
                        np.asarray(idx, dtype=np.int64), np.asarray(meas, dtype=np.int64),
                        np.asarray(vals, dtype=np.float64), **st)


def _vp(a):
    return None if a is None else a.ctypes.data


def _n_threads(B: int) -> int:
    return max(1, min(B // 8, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 1, 16))


def collate_ragged(r: RaggedEvents, padding_side: str = "right", do_produce_static_data: bool = True,
                   pin_memory: bool = False, n_threads: int | None = None) -> PytorchBatch:
    """Pads and tensorises the subjects of ``r`` into a CPU ``PytorchBatch`` (pinned if ``pin_memory``) through
    the native collate. Raises ``ValueError`` if the batch holds no dynamic element (as the reference does)."""
    if padding_side not in ("right", "left"):
        raise ValueError(f"seq_padding_side invalid: {padding_side}")
    lib = _lib.load(require_device=False)
    B = r.n_subjects
    if B == 0:
        raise ValueError("collate: empty batch")
    st_count = r.st_count if do_produce_static_data else None
    if do_produce_static_data and st_count is None:
        st_count = np.zeros(B, dtype=np.int64)
    L, M, S = (np.full(1, -1, np.int64) for _ in range(3))
    status = lib.esgpt_collate_shape(B, _vp(r.ev_start), _vp(r.ev_count), _vp(r.el_off), _vp(st_count),
                                     _vp(L), _vp(M), _vp(S))
    if status == _lib.ESGPT_ERR_INVALID_ARG and int(M[0]) == 0:
        raise ValueError("Batch has no dynamic measurements!")
    _lib.check(status, "esgpt_collate_shape")
    L, M, S = int(L[0]), int(M[0]), int(S[0])

    # every field a view into ONE (optionally pinned) buffer: the batch then moves to the device in one copy
    spec = {"event_mask": ((B, L), torch.bool), "time_delta": ((B, L), torch.float32),
            "dynamic_indices": ((B, L, M), torch.int64), "dynamic_measurement_indices": ((B, L, M), torch.int64),
            "dynamic_values": ((B, L, M), torch.float32), "dynamic_values_mask": ((B, L, M), torch.bool)}
    if do_produce_static_data:
        spec["static_indices"] = ((B, S), torch.int64)
        spec["static_measurement_indices"] = ((B, S), torch.int64)
    out = PytorchBatch.empty_packed(spec, pin_memory=pin_memory)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    st_args = ((_vp(r.st_start), _vp(st_count), _vp(r.st_idx), _vp(r.st_meas)) if do_produce_static_data and
               r.st_count is not None else (None, None, None, None))
    _lib.check(lib.esgpt_collate(
        B, _vp(r.ev_start), _vp(r.ev_count), _vp(r.time_delta), _vp(r.el_off), _vp(r.idx), _vp(r.meas),
        _vp(r.vals), *st_args, L, M, S if do_produce_static_data else 0, int(padding_side == "left"),
        p(out.event_mask), p(out.time_delta), p(out.dynamic_indices), p(out.dynamic_measurement_indices),
        p(out.dynamic_values), p(out.dynamic_values_mask), p(out.static_indices),
        p(out.static_measurement_indices), n_threads or _n_threads(B)), "esgpt_collate")
    return out


def collate(items: list[dict], padding_side: str = "right", do_produce_static_data: bool = True,
            pin_memory: bool = False) -> PytorchBatch:
    """``PytorchDataset.collate`` for a list of reference-format items (``pytorch_dataset.py:685-701``): the
    padded tensors, plus ``start_time`` / ``start_idx`` / ``end_idx`` / ``subject_id`` when the items hold them."""
    out = collate_ragged(flatten_items(items, do_produce_static_data), padding_side, do_produce_static_data,
                         pin_memory)
    if "start_time" in items[0]:
        out.start_time = torch.FloatTensor([e["start_time"] for e in items])
    for k in ("start_idx", "end_idx", "subject_id"):
        if k in items[0]:
            setattr(out, k, torch.LongTensor([e[k] for e in items]))
    return out


__all__ = ["RaggedEvents", "flatten_items", "collate_ragged", "collate"]
