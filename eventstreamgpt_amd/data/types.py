"""The batch contract of the training hot path.

Mirrors ``EventStream/data/types.py``: ``PytorchBatch`` (``:86-163``), ``DataModality`` (``:826-862``) and
``TemporalityType`` (``:802-823``). Field names, shapes and meanings are unchanged so a collated reference batch
can be handed to this package as-is.

One deliberate difference: the reference's ``__getitem__(str)`` goes through ``dataclasses.asdict`` and so
deep-copies every tensor on every string access (``types.py:251-258``; ~300 device copies per CI forward on a
GPU). Here string access returns the stored tensor itself. No hot-path code mutates a tensor obtained this way.
"""
from __future__ import annotations

import dataclasses
import enum
from typing import Any

import torch

from ..utils import StrEnum


class DataModality(StrEnum):
    """Modality of a measurement (``types.py:826-862``)."""

    DROPPED = enum.auto()
    SINGLE_LABEL_CLASSIFICATION = enum.auto()
    MULTI_LABEL_CLASSIFICATION = enum.auto()
    MULTIVARIATE_REGRESSION = enum.auto()
    UNIVARIATE_REGRESSION = enum.auto()


class TemporalityType(StrEnum):
    """How a measurement varies in time (``types.py:802-823``)."""

    STATIC = enum.auto()
    DYNAMIC = enum.auto()
    FUNCTIONAL_TIME_DEPENDENT = enum.auto()


_FLAT_ALIGN = 256

_TENSOR_FIELDS = (
    "event_mask",
    "time_delta",
    "time",
    "static_indices",
    "static_measurement_indices",
    "dynamic_indices",
    "dynamic_measurement_indices",
    "dynamic_values",
    "dynamic_values_mask",
    "start_time",
    "start_idx",
    "end_idx",
    "subject_id",
)


@dataclasses.dataclass
class PytorchBatch:
    """A collated batch of event streams.

    Shapes (B = subjects, L = events, M = data elements per event, S = static elements):
    ``event_mask`` bool [B,L]; ``time_delta`` f32 [B,L]; ``time`` f32 [B,L] (optional);
    ``static_indices`` / ``static_measurement_indices`` int64 [B,S]; ``dynamic_indices`` /
    ``dynamic_measurement_indices`` int64 [B,L,M]; ``dynamic_values`` f32 [B,L,M];
    ``dynamic_values_mask`` bool [B,L,M]. Index 0 is padding everywhere.
    """

    event_mask: torch.BoolTensor | None = None
    time_delta: torch.FloatTensor | None = None
    time: torch.FloatTensor | None = None
    static_indices: torch.LongTensor | None = None
    static_measurement_indices: torch.LongTensor | None = None
    dynamic_indices: torch.LongTensor | None = None
    dynamic_measurement_indices: torch.LongTensor | None = None
    dynamic_values: torch.FloatTensor | None = None
    dynamic_values_mask: torch.BoolTensor | None = None
    start_time: torch.FloatTensor | None = None
    start_idx: torch.LongTensor | None = None
    end_idx: torch.LongTensor | None = None
    subject_id: torch.LongTensor | None = None
    stream_labels: dict[str, torch.Tensor] | None = None

    @property
    def device(self) -> torch.device:
        return self.event_mask.device

    @property
    def batch_size(self) -> int:
        return self.event_mask.shape[0]

    @property
    def sequence_length(self) -> int:
        return self.event_mask.shape[1]

    @property
    def n_data_elements(self) -> int:
        return self.dynamic_indices.shape[2]

    @property
    def n_static_data_elements(self) -> int:
        return self.static_indices.shape[1]

    def keys(self):
        return [f.name for f in dataclasses.fields(self)]

    def values(self):
        return [getattr(self, k) for k in self.keys()]

    def items(self):
        return [(k, getattr(self, k)) for k in self.keys()]

    def get(self, item: str, default: Any) -> Any:
        return getattr(self, item) if item in self.keys() else default

    def __getitem__(self, item):
        if isinstance(item, str):
            if item not in self.keys():
                raise KeyError(item)
            return getattr(self, item)
        if isinstance(item, (tuple, int, slice)):
            return self._slice(item)
        raise TypeError(f"Invalid type {type(item)} for {item} for indexing!")

    def __setitem__(self, item: str, val: torch.Tensor):
        if not hasattr(self, item):
            raise KeyError(f"Key {item} not found")
        setattr(self, item, val)

    def _slice(self, index) -> "PytorchBatch":
        if not isinstance(index, tuple):
            index = (index,)
        if len(index) == 0 or len(index) > 3:
            raise ValueError(f"Invalid index {index} for PytorchBatch! Must be of length 1, 2, or 3.")
        b = index[0]
        s = index[1] if len(index) > 1 else slice(None)
        m = index[2] if len(index) > 2 else slice(None)

        def opt(t, *idx):
            return None if t is None else t[idx]

        return PytorchBatch(
            event_mask=self.event_mask[b, s],
            time_delta=opt(self.time_delta, b, s),
            time=opt(self.time, b, s),
            static_indices=opt(self.static_indices, b),
            static_measurement_indices=opt(self.static_measurement_indices, b),
            dynamic_indices=opt(self.dynamic_indices, b, s, m),
            dynamic_measurement_indices=opt(self.dynamic_measurement_indices, b, s, m),
            dynamic_values=opt(self.dynamic_values, b, s, m),
            dynamic_values_mask=opt(self.dynamic_values_mask, b, s, m),
            start_time=opt(self.start_time, b),
            start_idx=opt(self.start_idx, b),
            end_idx=opt(self.end_idx, b),
            subject_id=opt(self.subject_id, b),
            stream_labels=None if self.stream_labels is None else {k: v[b] for k, v in self.stream_labels.items()},
        )

    def last_sequence_element_unsqueezed(self) -> "PytorchBatch":
        """The last event of every subject, keeping a length-1 sequence dimension (``data/types.py:314-316``)."""
        return self[:, -1:]

    def repeat_batch_elements(self, expand_size: int) -> "PytorchBatch":
        """Each subject repeated ``expand_size`` times consecutively (``data/types.py:318-460``)."""
        idx = torch.arange(self.batch_size, device=self.device).repeat_interleave(expand_size)
        kw = {}
        for k in _TENSOR_FIELDS:
            v = getattr(self, k)
            kw[k] = None if v is None else v.index_select(0, idx)
        sl = self.stream_labels
        kw["stream_labels"] = None if sl is None else {k: v.index_select(0, idx) for k, v in sl.items()}
        return PytorchBatch(**kw)

    # ---- one-buffer layout: every tensor field a view into one flat byte buffer ----
    def flat_buffer(self) -> torch.Tensor | None:
        """The flat uint8 buffer every tensor field of this batch views, if it was built packed (``packed``,
        ``empty_packed`` or the native collate), else None. Staging such a batch is ONE copy (H2D or D2D)."""
        flat = getattr(self, "_flat", None)
        if flat is None:
            return None
        sig = getattr(self, "_flat_sig", ())
        for name, off, shape, dt in sig:  # still the views it was built with (fields may be reassigned)
            v = getattr(self, name)
            if (v is None or v.dtype != dt or tuple(v.shape) != shape or not v.is_contiguous()
                    or v.data_ptr() != flat.data_ptr() + off):
                return None
        return flat

    @staticmethod
    def empty_packed(spec: dict, device=None, pin_memory: bool = False) -> "PytorchBatch":
        """A batch whose fields ``spec`` = {name: (shape, dtype)} are views into one flat buffer (256-B aligned)."""
        sig, off = [], 0
        for name in _TENSOR_FIELDS:
            if name not in spec:
                continue
            shape, dt = tuple(spec[name][0]), spec[name][1]
            n = dt.itemsize
            for d in shape:
                n *= d
            sig.append((name, off, shape, dt))
            off += (n + _FLAT_ALIGN - 1) // _FLAT_ALIGN * _FLAT_ALIGN
        flat = torch.empty(max(off, 1), dtype=torch.uint8, device=device,
                           pin_memory=pin_memory and device in (None, "cpu") and torch.cuda.is_available())
        return PytorchBatch._from_flat(flat, tuple(sig))

    @staticmethod
    def _from_flat(flat: torch.Tensor, sig) -> "PytorchBatch":
        kw = {}
        for name, off, shape, dt in sig:
            n = dt.itemsize
            for d in shape:
                n *= d
            kw[name] = flat[off:off + n].view(dt).view(shape)
        out = PytorchBatch(**kw)
        out._flat, out._flat_sig = flat, sig
        return out

    def packed(self) -> "PytorchBatch":
        """A copy of this batch with every tensor field in one flat buffer on the same device (stream labels are
        copied into tensors of their own, so the copy never aliases this batch's labels)."""
        spec = {k: (tuple(v.shape), v.dtype) for k, v in self.as_dict().items()}
        out = PytorchBatch.empty_packed(spec, device=self.device)
        for k, v in self.as_dict().items():
            getattr(out, k).copy_(v)
        out.stream_labels = None if self.stream_labels is None else {k: v.clone() for k, v in self.stream_labels.items()}
        return out

    def shape_signature(self) -> tuple:
        """Names, shapes and dtypes of every tensor field and stream label: two batches with equal signatures can be
        staged into each other's buffers (``copy_``); a captured HIP graph replays only batches of its signature."""
        sig = tuple((k, tuple(v.shape), v.dtype) for k, v in self.as_dict().items())
        sl = self.stream_labels
        lab = () if sl is None else tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(sl.items()))
        return sig, lab

    def copy_(self, src: "PytorchBatch", non_blocking: bool = False) -> "PytorchBatch":
        """In-place copy of ``src``'s fields and stream labels: one buffer copy when both share a packed layout.
        Shapes must match exactly (no broadcasting: a size-1 dimension would silently duplicate entries)."""
        if self.shape_signature() != src.shape_signature():
            raise ValueError(f"PytorchBatch.copy_: shape signature mismatch\n  dst {self.shape_signature()}\n"
                             f"  src {src.shape_signature()}")
        a, b = self.flat_buffer(), src.flat_buffer()
        done = set()
        if a is not None and b is not None and self._flat_sig == src._flat_sig:
            a.copy_(b, non_blocking=non_blocking)
            done = {name for name, *_ in self._flat_sig}
        for k, v in src.as_dict().items():
            if k not in done:
                getattr(self, k).copy_(v, non_blocking=non_blocking)
        if src.stream_labels is not None:
            for k, v in src.stream_labels.items():
                self.stream_labels[k].copy_(v, non_blocking=non_blocking)
        return self

    def to(self, device, non_blocking: bool = False) -> "PytorchBatch":
        """Moves every tensor field to ``device`` (a packed batch moves as one buffer and stays packed)."""
        flat = self.flat_buffer()
        if flat is not None:
            out = PytorchBatch._from_flat(flat.to(device, non_blocking=non_blocking), self._flat_sig)
            packed = {name for name, *_ in self._flat_sig}
            for k, v in self.as_dict().items():  # fields set after packing travel on their own
                if k not in packed:
                    setattr(out, k, v.to(device, non_blocking=non_blocking))
            sl = self.stream_labels
            out.stream_labels = None if sl is None else {k: v.to(device) for k, v in sl.items()}
            return out
        kw = {}
        for k in _TENSOR_FIELDS:
            v = getattr(self, k)
            kw[k] = None if v is None else v.to(device, non_blocking=non_blocking)
        sl = self.stream_labels
        kw["stream_labels"] = None if sl is None else {k: v.to(device) for k, v in sl.items()}
        return PytorchBatch(**kw)

    def as_dict(self) -> dict[str, torch.Tensor]:
        return {k: getattr(self, k) for k in _TENSOR_FIELDS if getattr(self, k) is not None}
