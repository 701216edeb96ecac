"""``PytorchDataset`` over the cached deep-learning representation (``DL_reps/{split}*.parquet``), without polars.

Mirrors ``EventStream/data/pytorch_dataset.py`` (``PytorchDataset``: ``__init__`` ``:118-300``,
``_build_task_cached_df`` ``:390-425``, ``__len__`` / ``__getitem__`` / ``_seeded_getitem`` ``:437-525``,
``collate`` ``:685-701``) and ``PytorchDatasetConfig`` (``EventStream/data/config.py:650-790``).

Layout. The reference keeps a polars frame and converts it to Python rows (``.rows()``), then pads each item
event by event at collate time. Here the parquet columns are read with pyarrow straight into one flat store
(``RaggedEvents``): per-event ``time_delta`` / element offsets and per-element index / measurement / value arrays
for the whole split, int64/float64, contiguous. A sampled item is a window (first event, count) into that store;
``batch`` samples the windows for a set of subjects and hands them to the native collate, which writes the padded
batch into pinned host memory in one pass. ``__getitem__`` + ``collate`` keep the reference's item-dict API.

Deliberate differences (documented in DESIGN.md):
* ``train_subset_size`` draws the subset with numpy's ``default_rng(train_subset_seed)``, not polars' sampler
  (the chosen subjects differ for the same seed; the subset size is the same);
* the task-restricted representation is built in memory and not cached under ``DL_reps/for_task`` (the
  reference writes it there; its own re-load glob never matches, ``pytorch_dataset.py:156``);
* ``start_time`` minutes use UTC epoch seconds (the reference calls ``datetime.timestamp()`` on a naive datetime,
  i.e. host local time);
* null and NaN values are both NaN in the store (``collate`` treats them identically).
"""
from __future__ import annotations

import dataclasses
import enum
import glob
import json
import math
from pathlib import Path

import numpy as np
import torch

from ..utils import StrEnum
from .collate import RaggedEvents, collate, collate_ragged
from .types import PytorchBatch


class SeqPaddingSide(StrEnum):
    """``config.py:607-620``."""

    RIGHT = enum.auto()
    LEFT = enum.auto()


class SubsequenceSamplingStrategy(StrEnum):
    """``config.py:623-647``."""

    TO_END = enum.auto()
    FROM_START = enum.auto()
    RANDOM = enum.auto()


@dataclasses.dataclass
class PytorchDatasetConfig:
    """``PytorchDatasetConfig`` (``config.py:650-790``): same fields, defaults and validation."""

    save_dir: Path | str | None = None
    max_seq_len: int = 256
    min_seq_len: int = 2
    seq_padding_side: SeqPaddingSide = SeqPaddingSide.RIGHT
    subsequence_sampling_strategy: SubsequenceSamplingStrategy = SubsequenceSamplingStrategy.RANDOM
    train_subset_size: int | float | str = "FULL"
    train_subset_seed: int | None = None
    task_df_name: str | None = None
    do_include_subsequence_indices: bool = False
    do_include_subject_id: bool = False
    do_include_start_time_min: bool = False

    def __post_init__(self):
        if self.seq_padding_side not in SeqPaddingSide.values():
            raise ValueError(f"seq_padding_side invalid; must be in {', '.join(SeqPaddingSide.values())}")
        self.seq_padding_side = SeqPaddingSide(self.seq_padding_side)
        if self.subsequence_sampling_strategy not in SubsequenceSamplingStrategy.values():
            raise ValueError(f"Invalid subsequence_sampling_strategy {self.subsequence_sampling_strategy}")
        self.subsequence_sampling_strategy = SubsequenceSamplingStrategy(self.subsequence_sampling_strategy)
        if not (isinstance(self.min_seq_len, int) and self.min_seq_len >= 0):
            raise ValueError(f"min_seq_len must be a non-negative integer; got {self.min_seq_len}")
        if not (isinstance(self.max_seq_len, int) and self.max_seq_len >= self.min_seq_len):
            raise ValueError(f"max_seq_len must be an integer at least equal to min_seq_len; got {self.max_seq_len} "
                             f"(min {self.min_seq_len})")
        if isinstance(self.save_dir, str):
            self.save_dir = Path(self.save_dir)
        match self.train_subset_size:
            case int() as n if n < 0:
                raise ValueError(f"If integral, train_subset_size must be positive! Got {n}")
            case float() as frac if frac <= 0 or frac >= 1:
                raise ValueError(f"If float, train_subset_size must be in (0, 1)! Got {frac}")
            case int() | float() if self.train_subset_seed is None:
                self.train_subset_seed = int(np.random.randint(1, int(1e6)))
            case None | "FULL" | int() | float():
                pass
            case _:
                raise TypeError(f"train_subset_size is of unrecognized type {type(self.train_subset_size)}.")


# ---- parquet -> flat arrays -----------------------------------------------------------------------------------

def _ranges(starts: np.ndarray, counts: np.ndarray) -> np.ndarray:
    """Concatenation of ``arange(s, s + c)`` over the pairs, vectorised."""
    counts = np.asarray(counts, dtype=np.int64)
    total = int(counts.sum())
    if total == 0:
        return np.zeros(0, dtype=np.int64)
    rep = np.repeat(np.asarray(starts, dtype=np.int64) - np.concatenate([[0], np.cumsum(counts)[:-1]]), counts)
    return rep + np.arange(total, dtype=np.int64)


def _lengths(arr) -> np.ndarray:
    import pyarrow.compute as pc

    return np.asarray(pc.fill_null(pc.list_value_length(arr), 0).to_numpy(zero_copy_only=False), dtype=np.int64)


def _num(arr, dtype, fill) -> np.ndarray:
    import pyarrow.compute as pc

    if len(arr) == 0:
        return np.zeros(0, dtype=dtype)
    return np.asarray(pc.fill_null(arr.cast("float64" if dtype == np.float64 else "int64"), fill)
                      .to_numpy(zero_copy_only=False), dtype=dtype)


@dataclasses.dataclass
class _Store:
    """The split as flat arrays (what the reader loads before any filtering)."""

    subject_id: np.ndarray          # [n] int64
    start_time_min: np.ndarray      # [n] float64, minutes since the UNIX epoch
    n_events: np.ndarray            # [n] int64 (-1: null sequence)
    ev_start: np.ndarray            # [n] int64
    time: np.ndarray | None         # [E] float64 minutes since start_time (DL_reps `time`)
    time_delta: np.ndarray | None   # [E] float64 (already-converted DL_reps with a `time_delta` column)
    el_off: np.ndarray              # [E+1]
    idx: np.ndarray                 # [nnz] int64
    meas: np.ndarray                # [nnz] int64
    vals: np.ndarray                # [nnz] float64 (NaN: missing)
    st_start: np.ndarray | None
    st_count: np.ndarray | None
    st_idx: np.ndarray | None
    st_meas: np.ndarray | None
    labels: dict[str, np.ndarray]


def _read_dl_reps(files: list[str], label_columns=()) -> _Store:
    """Reads DL_reps parquet shards (format: ``dataset_base.py:1063-1122``) into a ``_Store``."""
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.parquet as pq

    if not files:
        raise FileNotFoundError("no DL_reps parquet files")
    tables = [pq.read_table(f) for f in files]
    cols = tables[0].column_names

    def column(name):
        chunks = []
        for t in tables:
            c = t.column(name)
            chunks.extend(c.chunks)
        typ = chunks[0].type
        if any(ch.type != typ for ch in chunks):  # shards written with different widths (uint8 vs uint16 ...)
            if pa.types.is_list(typ) or pa.types.is_large_list(typ):
                typ = _widen(typ)
            chunks = [ch.cast(typ) for ch in chunks]
        return pa.chunked_array(chunks, type=typ).combine_chunks()

    sid = _num(column("subject_id"), np.int64, 0)
    n = sid.shape[0]
    st = column("start_time")
    st_us = np.asarray(st.cast(pa.timestamp("us")).cast(pa.int64()).to_numpy(zero_copy_only=False), dtype=np.float64)
    start_time_min = st_us / 6e7

    di = column("dynamic_indices")
    null_seq = np.asarray(di.is_null().to_numpy(zero_copy_only=False), dtype=bool)
    n_events = _lengths(di)
    ev_start = np.concatenate([[0], np.cumsum(n_events)[:-1]]) if n else np.zeros(0, np.int64)
    ev_idx = di.flatten()                    # one entry per event of the non-null subjects
    el_len = _lengths(ev_idx)
    el_off = np.concatenate([[0], np.cumsum(el_len)]).astype(np.int64)
    idx = _num(ev_idx.flatten(), np.int64, 0)
    E, nnz = el_len.shape[0], idx.shape[0]

    dm = column("dynamic_measurement_indices")
    meas = _aligned_elements(dm, n_events, null_seq, el_len, np.int64, 0)
    dv = column("dynamic_values")
    vals = _aligned_elements(dv, n_events, null_seq, el_len, np.float64, math.nan)

    time = time_delta = None
    if "time" in cols:
        tm = column("time")
        if not np.array_equal(_lengths(tm)[~null_seq], n_events[~null_seq]):
            raise ValueError("DL_reps: time and dynamic_indices disagree on event counts")
        time = _aligned_events(tm, n_events, null_seq)
    elif "time_delta" in cols:  # already converted: used as is (pytorch_dataset.py:247)
        time_delta = _aligned_events(column("time_delta"), n_events, null_seq)
    else:
        raise ValueError("DL_reps: neither `time` nor `time_delta` is present")
    n_events = np.where(null_seq, -1, n_events)

    st_start = st_count = st_idx = st_meas = None
    if "static_indices" in cols:
        si, sm = column("static_indices"), column("static_measurement_indices")
        st_count = _lengths(si)
        st_start = np.concatenate([[0], np.cumsum(st_count)[:-1]]) if n else np.zeros(0, np.int64)
        st_idx = _num(si.flatten(), np.int64, 0)
        st_meas = _num(sm.flatten(), np.int64, 0)
        if not np.array_equal(_lengths(sm), st_count):
            raise ValueError("DL_reps: static_indices and static_measurement_indices disagree on lengths")
    labels = {c: column(c) for c in label_columns}
    assert idx.shape[0] == nnz and el_off.shape[0] == E + 1
    del pc
    return _Store(sid, start_time_min, n_events, ev_start, time, time_delta, el_off, idx, meas, vals, st_start, st_count,
                  st_idx, st_meas, labels)


def _widen(typ):
    import pyarrow as pa

    if pa.types.is_list(typ) or pa.types.is_large_list(typ):
        return pa.large_list(_widen(typ.value_type))
    if pa.types.is_integer(typ):
        return pa.int64()
    if pa.types.is_floating(typ):
        return pa.float64()
    return typ


def _aligned_events(col, n_events, null_seq) -> np.ndarray:
    """Per-event float64 array of a list<double> column aligned to the dynamic_indices events (null subject:
    NaN for each of its events)."""
    out = np.full(int(n_events[~null_seq].sum()) if n_events.size else 0, math.nan)
    has = ~np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool) & ~null_seq
    lens = _lengths(col)
    flat = _num(col.flatten(), np.float64, math.nan)
    ev_start = np.concatenate([[0], np.cumsum(np.where(null_seq, 0, n_events))[:-1]]) if n_events.size else n_events
    src_start = np.concatenate([[0], np.cumsum(lens)[:-1]]) if lens.size else lens
    take = has & (lens == np.where(null_seq, 0, n_events))
    out[_ranges(ev_start[take], n_events[take])] = flat[_ranges(src_start[take], lens[take])]
    return out


def _aligned_elements(col, n_events, null_seq, el_len, dtype, fill) -> np.ndarray:
    """Per-element array of a list<list<x>> column aligned to the dynamic_indices elements. A null subject list,
    a null event list or a null element reads as ``fill``; lists whose lengths disagree with dynamic_indices
    raise (the reference's collate would pad them inconsistently)."""
    import pyarrow.compute as pc

    nnz = int(el_len.sum())
    out = np.full(nnz, fill, dtype=dtype)
    subj_has = ~np.asarray(col.is_null().to_numpy(zero_copy_only=False), dtype=bool) & ~null_seq
    subj_len = _lengths(col)
    n_ev = np.where(null_seq, 0, n_events)
    if not np.array_equal(subj_len[subj_has], n_ev[subj_has]):
        raise ValueError("DL_reps: a dynamic column disagrees with dynamic_indices on event counts")
    events = col.flatten()                                    # events of the subjects with a non-null list
    ev_has = ~np.asarray(events.is_null().to_numpy(zero_copy_only=False), dtype=bool)
    ev_len = _lengths(events)
    # position of each of these events among the dynamic_indices events
    subj_ev_start = np.concatenate([[0], np.cumsum(n_ev)[:-1]]) if n_ev.size else n_ev
    ev_pos = _ranges(subj_ev_start[subj_has], n_ev[subj_has])
    if not np.array_equal(ev_len[ev_has], el_len[ev_pos[ev_has]]):
        raise ValueError("DL_reps: a dynamic column disagrees with dynamic_indices on element counts")
    el_start = np.concatenate([[0], np.cumsum(el_len)[:-1]]) if el_len.size else el_len
    dst = _ranges(el_start[ev_pos[ev_has]], ev_len[ev_has])
    flat = events.flatten()
    vals = np.asarray(pc.fill_null(flat.cast("float64" if dtype == np.float64 else "int64"), fill)
                      .to_numpy(zero_copy_only=False), dtype=dtype) if len(flat) else np.zeros(0, dtype=dtype)
    out[dst] = vals
    return out


def _normalize_task(arr):
    """``PytorchDataset.normalize_task`` (``pytorch_dataset.py:94-116``) over an Arrow column: integers ->
    multi-class (as is), dictionary / string -> multi-class codes (in order of first appearance, like a polars
    Categorical's physical codes), booleans -> binary (float32), floats -> regression."""
    import pyarrow as pa

    t = arr.type
    if pa.types.is_integer(t):
        return "multi_class_classification", np.asarray(arr.to_numpy(zero_copy_only=False), dtype=np.int64)
    if pa.types.is_dictionary(t) or pa.types.is_string(t) or pa.types.is_large_string(t):
        vals = arr.to_pylist()
        codes, out = {}, []
        for v in vals:
            out.append(codes.setdefault(v, len(codes)))
        return "multi_class_classification", np.asarray(out, dtype=np.int64)
    if pa.types.is_boolean(t):
        return "binary_classification", np.asarray(arr.to_numpy(zero_copy_only=False), dtype=np.float32)
    if pa.types.is_floating(t):
        return "regression", np.asarray(arr.to_numpy(zero_copy_only=False), dtype=np.float64)
    raise TypeError(f"Can't process label of {t} type!")


class PytorchDataset(torch.utils.data.Dataset):
    """``PytorchDataset`` (``pytorch_dataset.py:57-701``) on the flat store.

    Attributes as in the reference: ``config``, ``split``, ``vocabulary_config`` (dict), ``measurement_configs``
    (dict of JSON dicts, dropped ones removed), ``has_task``, ``tasks``, ``task_types``, ``task_vocabs``,
    ``do_produce_static_data``, ``seq_padding_side``, ``max_seq_len``, ``mean_log_inter_event_time_min``,
    ``std_log_inter_event_time_min``, ``subject_ids``.
    """

    def __init__(self, config: PytorchDatasetConfig, split: str):
        super().__init__()
        self.config = config
        self.split = split
        self.task_types: dict[str, str] = {}
        self.task_vocabs: dict[str, list] = {}
        save_dir = Path(config.save_dir)
        with open(save_dir / "vocabulary_config.json") as f:
            self.vocabulary_config = json.load(f)
        with open(save_dir / "inferred_measurement_configs.json") as f:
            mcs = json.load(f)
        self.measurement_configs = {k: v for k, v in mcs.items() if v.get("modality") != "dropped"}

        files = sorted(glob.glob(str(save_dir / "DL_reps" / f"{split}*.parquet")))
        store = _read_dl_reps(files)
        ev_lo = ev_n = None
        if config.task_df_name is not None:
            raw = save_dir / "task_dfs" / f"{config.task_df_name}.parquet"
            if not raw.is_file():
                raise FileNotFoundError(f"{raw} does not exist, but config.task_df_name = {config.task_df_name}!")
            rows, ev_lo, ev_n = self._restrict_to_task(store, raw)
            self.has_task = True
        else:
            rows = np.arange(store.subject_id.shape[0])
            self.has_task = False
            self.tasks = None
            self.task_vocabs = None
        self._store = store
        self.do_produce_static_data = store.st_count is not None
        self.seq_padding_side = config.seq_padding_side
        self.max_seq_len = config.max_seq_len

        # per-row windows into the store's events
        first = store.ev_start[rows] + (0 if ev_lo is None else ev_lo)
        count = np.where(store.n_events[rows] < 0, -1, store.n_events[rows] if ev_n is None else ev_n)
        keep = count >= config.min_seq_len  # (a null list has no length: dropped, like polars' filter)
        rows, first, count = rows[keep], first[keep], count[keep]
        if ev_lo is not None:
            self._labels = {k: v[keep] for k, v in self._labels.items()}

        # time -> time_delta (next - this, the last event 1: pytorch_dataset.py:247-259); start_time += time[0]
        ev = _ranges(first, count)
        ends = np.cumsum(count) - 1
        starts_new = np.concatenate([[0], ends[:-1] + 1]).astype(np.int64) if count.size else count
        if store.time is not None:
            t = store.time[ev]
            td = np.empty_like(t)
            td[:-1] = t[1:] - t[:-1]
            td[ends] = 1.0
            start_time = store.start_time_min[rows] + (t[starts_new] if count.size else 0.0)
        else:
            td = store.time_delta[ev]
            start_time = store.start_time_min[rows]

        # inter-event-time stats over every delta (:262-287), then drop subjects with a delta <= 0
        with np.errstate(divide="ignore", invalid="ignore"):
            logs = np.log(td)
        self.mean_log_inter_event_time_min = float(logs.mean()) if logs.size else math.nan
        self.std_log_inter_event_time_min = float(logs.std(ddof=1)) if logs.size > 1 else math.nan
        if td.size and td.min() <= 0:
            bad = np.minimum.reduceat(td, starts_new) <= 0
            print(f"WARNING: Observed inter-event times <= 0 for {int(bad.sum())} subjects! Removing malformed "
                  "subjects")
            ok = ~bad
            sel = np.repeat(ok, count)
            rows, first, count, start_time = rows[ok], first[ok], count[ok], start_time[ok]
            ev, td = ev[sel], td[sel]
            if ev_lo is not None:
                self._labels = {k: v[ok] for k, v in self._labels.items()}

        if config.train_subset_size not in (None, "FULL") and split == "train":
            n = rows.shape[0]
            k = config.train_subset_size if isinstance(config.train_subset_size, int) else \
                int(n * config.train_subset_size)
            pick = np.sort(np.random.default_rng(config.train_subset_seed).choice(n, size=min(k, n), replace=False))
            sel = np.repeat(np.isin(np.arange(n), pick), count)
            rows, first, count, start_time = rows[pick], first[pick], count[pick], start_time[pick]
            ev, td = ev[sel], td[sel]
            if ev_lo is not None:
                self._labels = {k2: v[pick] for k2, v in self._labels.items()}

        # the dataset's own event arrays: gathered once (windows are contiguous in the store already, but a task
        # restriction changes the last delta, so time_delta is per dataset); elements stay shared
        ev_start = np.concatenate([[0], np.cumsum(count)[:-1]]).astype(np.int64) if count.size else count
        el_len = (store.el_off[1:] - store.el_off[:-1])[ev]
        el_src = store.el_off[:-1][ev]
        self.subject_ids = store.subject_id[rows].tolist()
        self.start_time_min = start_time
        el = _ranges(el_src, el_len)
        self.events = RaggedEvents(
            ev_start, count, td, np.concatenate([[0], np.cumsum(el_len)]), store.idx[el], store.meas[el],
            store.vals[el],
            None if store.st_count is None else store.st_start[rows],
            None if store.st_count is None else store.st_count[rows], store.st_idx, store.st_meas)

    # ---- task restriction (_build_task_cached_df, :390-425) ---------------------------------------------------
    def _restrict_to_task(self, store: _Store, task_fp: Path):
        import pyarrow.parquet as pq

        if store.time is None:
            raise NotImplementedError("task restriction needs a DL_reps `time` column")
        task = pq.read_table(task_fp)
        tsid = np.asarray(task.column("subject_id").to_numpy(), dtype=np.int64)
        import pyarrow as pa

        def minutes(c):
            return np.asarray(task.column(c).cast(pa.timestamp("us")).cast(pa.int64()).to_numpy(), np.float64) / 6e7

        t_start, t_end = minutes("start_time"), minutes("end_time")
        self.tasks = sorted(c for c in task.column_names if c not in ("subject_id", "start_time", "end_time"))
        labels = {}
        for c in self.tasks:
            typ, vals = _normalize_task(task.column(c).combine_chunks())
            self.task_types[c] = typ
            labels[c] = vals
            if typ == "binary_classification":
                self.task_vocabs[c] = [False, True]
            elif typ == "multi_class_classification":
                self.task_vocabs[c] = list(range(int(vals.max()) if vals.size else 0))
        rows, lo, cnt, pick = [], [], [], []
        by_sid = {}
        for j, s in enumerate(tsid):
            by_sid.setdefault(int(s), []).append(j)
        for r, s in enumerate(store.subject_id):       # inner join, left (cached data) order
            for j in by_sid.get(int(s), []):
                rows.append(r)
                pick.append(j)
                n = store.n_events[r]
                if n < 0:
                    lo.append(0)
                    cnt.append(-1)
                    continue
                t = store.time[store.ev_start[r]:store.ev_start[r] + n]
                a = int(np.searchsorted(t, t_start[j] - store.start_time_min[r], side="left"))
                b = int(np.searchsorted(t, t_end[j] - store.start_time_min[r], side="left"))
                lo.append(a)
                cnt.append(max(0, b - a))
        pick = np.asarray(pick, dtype=np.int64)
        self._labels = {c: v[pick] for c, v in labels.items()}
        return np.asarray(rows, np.int64), np.asarray(lo, np.int64), np.asarray(cnt, np.int64)

    # ---- item API -----------------------------------------------------------------------------------------------
    def __len__(self) -> int:
        return self.events.n_subjects

    def _window(self, idx: int, rng=None) -> tuple[int, int]:
        n = int(self.events.ev_count[idx])
        if n <= self.max_seq_len:
            return 0, n
        match self.config.subsequence_sampling_strategy:
            case SubsequenceSamplingStrategy.RANDOM:
                st = int(np.random.choice(n - self.max_seq_len)) if rng is None else \
                    int(rng.integers(0, n - self.max_seq_len))
            case SubsequenceSamplingStrategy.TO_END:
                st = n - self.max_seq_len
            case SubsequenceSamplingStrategy.FROM_START:
                st = 0
            case _:
                raise ValueError(f"Invalid sampling strategy: {self.config.subsequence_sampling_strategy}!")
        return st, self.max_seq_len

    def __getitem__(self, idx: int) -> dict:
        return self._seeded_getitem(idx)

    def _seeded_getitem(self, idx: int, seed: int | None = None) -> dict:
        """``_seeded_getitem`` (``:473-525``): the subject's data as Python lists, cut to ``max_seq_len`` events.
        ``seed`` seeds numpy's global RNG first, as the reference's ``SeedableMixin.WithSeed`` does."""
        if seed is not None:
            np.random.seed(seed)
        r = self.events
        st, n = self._window(idx)
        a = int(r.ev_start[idx]) + st
        item = {}
        if self.do_produce_static_data:
            s0, sc = int(r.st_start[idx]), int(r.st_count[idx])
            item["static_indices"] = r.st_idx[s0:s0 + sc].tolist()
            item["static_measurement_indices"] = r.st_meas[s0:s0 + sc].tolist()
        item["time_delta"] = r.time_delta[a:a + n].tolist()
        off = r.el_off[a:a + n + 1]
        e0, e1 = int(off[0]), int(off[-1])
        cuts = (off[1:-1] - e0).tolist()
        item["dynamic_indices"] = [x.tolist() for x in np.split(r.idx[e0:e1], cuts)]
        item["dynamic_measurement_indices"] = [x.tolist() for x in np.split(r.meas[e0:e1], cuts)]
        item["dynamic_values"] = [[None if math.isnan(v) else v for v in x.tolist()]
                                  for x in np.split(r.vals[e0:e1], cuts)]
        if self.config.do_include_subject_id:
            item["subject_id"] = self.subject_ids[idx]
        if self.config.do_include_start_time_min:
            item["start_time"] = float(self.start_time_min[idx] + r.time_delta[r.ev_start[idx]:a].sum())
        if self.config.do_include_subsequence_indices:
            item["start_idx"], item["end_idx"] = st, st + n
        if self.has_task:
            for t in self.tasks:
                v = self._labels[t][idx]
                item[t] = v.item()
        return item

    def collate(self, batch: list[dict]) -> PytorchBatch:
        """``collate`` (``:685-701``) through the native collate."""
        out = collate(batch, str(self.seq_padding_side), self.do_produce_static_data)
        if self.has_task:
            out.stream_labels = {t: self._label_tensor(t, [e[t] for e in batch]) for t in self.tasks}
        return out

    def _label_tensor(self, task, vals):
        match self.task_types[task]:
            case "multi_class_classification":
                return torch.LongTensor(vals)
            case "binary_classification" | "regression":
                return torch.FloatTensor(vals)
            case t:
                raise TypeError(f"Don't know how to tensorify task of type {t}!")

    # ---- native batch path --------------------------------------------------------------------------------------
    def batch(self, indices, rng: np.random.Generator | None = None, pin_memory: bool = False) -> PytorchBatch:
        """Samples each subject's window (the configured strategy; ``rng`` draws the RANDOM starts) and collates
        the windows straight from the flat store: no per-item Python lists."""
        indices = np.asarray(indices, dtype=np.int64)
        r = self.events
        n = r.ev_count[indices]
        over = np.maximum(n - self.max_seq_len, 0)
        match self.config.subsequence_sampling_strategy:
            case SubsequenceSamplingStrategy.RANDOM:
                g = rng if rng is not None else np.random.default_rng()
                st = np.where(over > 0, g.integers(0, np.maximum(over, 1)), 0)
            case SubsequenceSamplingStrategy.TO_END:
                st = over
            case _:
                st = np.zeros_like(over)
        out = collate_ragged(r.window(indices, st, np.minimum(n, self.max_seq_len)), str(self.seq_padding_side),
                             self.do_produce_static_data, pin_memory)
        if self.config.do_include_subject_id:
            out.subject_id = torch.as_tensor(np.asarray(self.subject_ids)[indices], dtype=torch.long)
        if self.config.do_include_start_time_min:
            pre = np.array([r.time_delta[r.ev_start[i]:r.ev_start[i] + s].sum() for i, s in zip(indices, st)])
            out.start_time = torch.as_tensor(self.start_time_min[indices] + pre, dtype=torch.float32)
        if self.config.do_include_subsequence_indices:
            out.start_idx = torch.as_tensor(st, dtype=torch.long)
            out.end_idx = torch.as_tensor(st + np.minimum(n, self.max_seq_len), dtype=torch.long)
        if self.has_task:
            out.stream_labels = {t: self._label_tensor(t, self._labels[t][indices].tolist()) for t in self.tasks}
        return out

    def batches(self, batch_size: int, shuffle: bool = True, seed: int = 0, drop_last: bool = False,
                pin_memory: bool = False, rank: int = 0, world_size: int = 1):
        """Epoch iterator over native batches. With ``world_size`` > 1 each rank takes a disjoint stride of the
        (shared-seed) permutation, as ``DistributedSampler`` does."""
        g = np.random.default_rng(seed)
        order = g.permutation(len(self)) if shuffle else np.arange(len(self))
        order = order[rank::world_size]
        for i in range(0, order.shape[0], batch_size):
            sel = order[i:i + batch_size]
            if drop_last and sel.shape[0] < batch_size:
                break
            yield self.batch(sel, g, pin_memory)


__all__ = ["PytorchDataset", "PytorchDatasetConfig", "SeqPaddingSide", "SubsequenceSamplingStrategy"]
