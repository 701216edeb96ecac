"""Batch producer: the native collate and the DL_reps reader against the reference.

Host code only (no GPU): the C++ collate lives in libesgpt_amd.so and runs on the host, so these tests need the
built library but not a device. Checked against
* the reference tests' known answers (``tests/golden/collate_known_answers.json``, ``dl_reps_known_answers.json``:
  ``tests/data/test_pytorch_dataset.py:27-300,402-830``),
* what the reference ``PytorchDataset.collate`` returned on seeded random ragged batches (``collate_ref.pt``,
  made by ``tests/golden/make_collate_golden.py``),
* the oracle restatement (``oracle/collate_oracle.py``) on larger random batches and on the reference's sample
  DL_reps shard (``tests/golden/sample_dl_reps``, copied from ``sample_data/processed/sample``).
"""
import json
import math
import os
from datetime import datetime

import numpy as np
import pytest
import torch

from eventstreamgpt_amd import _lib

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIELDS = ("event_mask", "time_delta", "dynamic_indices", "dynamic_measurement_indices", "dynamic_values",
          "dynamic_values_mask", "static_indices", "static_measurement_indices")

pytestmark = pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="library not built")


def _eq(got, want, what):
    assert got.dtype == want.dtype, (what, got.dtype, want.dtype)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    assert torch.equal(got, want), what


def test_collate_known_answers():
    from eventstreamgpt_amd.data.collate import collate
    import collate_oracle as O

    ka = json.load(open(os.path.join(GOLDEN, "collate_known_answers.json")))
    for c in ka["cases"]:
        got = collate(c["items"], c["padding"], c["static"])
        ora = O.collate(c["items"], c["padding"], c["static"])
        for k, w in c["want"].items():
            g = getattr(got, k)
            want = torch.tensor(w, dtype=g.dtype)
            _eq(g, want, (c["name"], k))
            _eq(ora[k], want, (c["name"], k, "oracle"))
        if not c["static"]:
            assert got.static_indices is None


def test_collate_matches_reference_outputs():
    from eventstreamgpt_amd.data.collate import collate

    for c in torch.load(os.path.join(GOLDEN, "collate_ref.pt"), weights_only=True):
        items = json.loads(c["items_json"])
        got = collate(items, c["padding"], c["static"])
        for k, w in c["want"].items():
            _eq(getattr(got, k), w, (c["name"], k))


def _random_items(rng, B, L, M, S, vmax=1210):
    items = []
    for _ in range(B):
        n = int(rng.integers(1, L + 1))
        it = {"time_delta": rng.exponential(20.0, n).tolist(), "dynamic_indices": [],
              "dynamic_measurement_indices": [], "dynamic_values": []}
        for _ in range(n):
            k = int(rng.integers(0, M + 1))
            it["dynamic_indices"].append(rng.integers(1, vmax, k).tolist())
            it["dynamic_measurement_indices"].append(rng.integers(1, 5, k).tolist())
            v = rng.normal(0, 1, k)
            v[rng.random(k) < 0.4] = np.nan
            it["dynamic_values"].append([None if math.isnan(x) else x for x in v.tolist()])
        s = int(rng.integers(0, S + 1))
        it["static_indices"] = rng.integers(1, 9, s).tolist()
        it["static_measurement_indices"] = [1] * s
        items.append(it)
    return items


@pytest.mark.parametrize("side", ["right", "left"])
@pytest.mark.parametrize("threads", [1, 5])
def test_collate_vs_oracle_random(side, threads):
    from eventstreamgpt_amd.data.collate import collate_ragged, flatten_items
    import collate_oracle as O

    rng = np.random.default_rng(7 + threads)
    items = _random_items(rng, 40, 64, 16, 3)
    got = collate_ragged(flatten_items(items), side, True, n_threads=threads)
    ora = O.collate(items, side, True)
    for k in FIELDS:
        _eq(getattr(got, k), ora[k], k)


def test_collate_edge_cases():
    from eventstreamgpt_amd.data.collate import RaggedEvents, collate, collate_ragged

    # no dynamic element anywhere: the reference's ValueError
    with pytest.raises(ValueError, match="no dynamic measurements"):
        collate([{"time_delta": [1.0], "dynamic_indices": [[]], "dynamic_measurement_indices": [[]],
                  "dynamic_values": [[]], "static_indices": [], "static_measurement_indices": []}])
    # all-empty static lists -> S = 0; NaN time delta -> masked event; a None value list -> all values missing
    out = collate([{"time_delta": [1.0, float("nan")], "dynamic_indices": [[3, 4], [5]],
                    "dynamic_measurement_indices": [[1, 2], [2]], "dynamic_values": [None, [2.5]],
                    "static_indices": [], "static_measurement_indices": []}])
    assert out.static_indices.shape == (1, 0)
    assert out.event_mask.tolist() == [[True, False]]
    assert out.dynamic_values_mask.tolist() == [[[False, False], [True, False]]]
    assert out.dynamic_values.tolist() == [[[0.0, 0.0], [2.5, 0.0]]]
    # indices beyond float32's exact range stay exact (the reference's float32 round trip would round them)
    big = 2 ** 40 + 3
    out = collate([{"time_delta": [1.0], "dynamic_indices": [[big]], "dynamic_measurement_indices": [[1]],
                    "dynamic_values": [[None]], "static_indices": [big], "static_measurement_indices": [1]}])
    assert out.dynamic_indices.item() == big and out.static_indices.item() == big
    # shape mismatches are rejected by the ABI, not written out of bounds
    r = RaggedEvents([0], [2], [1.0, 1.0], [0, 1, 3], [1, 2, 3], [1, 1, 1], [0.0] * 3)
    lib = _lib.load(require_device=False)
    buf = np.zeros(64, np.int64)
    p = buf.ctypes.data
    assert lib.esgpt_collate(1, r.ev_start.ctypes.data, r.ev_count.ctypes.data, r.time_delta.ctypes.data,
                             r.el_off.ctypes.data, r.idx.ctypes.data, r.meas.ctypes.data, r.vals.ctypes.data,
                             None, None, None, None, 2, 1, 0, 0, p, p, p, p, p, p, None, None, 1) \
        == _lib.ESGPT_ERR_INVALID_ARG
    assert collate_ragged(r).dynamic_indices.tolist() == [[[1, 0], [2, 3]]]
    with pytest.raises(ValueError):
        collate_ragged(r, "middle")


def _write_known_frame(d):
    import pyarrow as pa
    import pyarrow.parquet as pq

    ka = json.load(open(os.path.join(GOLDEN, "dl_reps_known_answers.json")))
    f = ka["frame"]
    os.makedirs(os.path.join(d, "DL_reps"), exist_ok=True)
    ts = lambda m: [None if x is None else datetime.utcfromtimestamp(x * 60) for x in m]  # noqa: E731
    u64l = pa.list_(pa.uint64())
    tbl = pa.table({
        "subject_id": pa.array(f["subject_id"], pa.uint8()),
        "start_time": pa.array(ts(f["start_time_min"]), pa.timestamp("us")),
        "time": pa.array(f["time"], pa.list_(pa.float64())),
        "static_indices": pa.array(f["static_indices"], u64l),
        "static_measurement_indices": pa.array(f["static_measurement_indices"], u64l),
        "dynamic_indices": pa.array(f["dynamic_indices"], pa.list_(u64l)),
        "dynamic_measurement_indices": pa.array(f["dynamic_measurement_indices"], pa.list_(u64l)),
        "dynamic_values": pa.array(f["dynamic_values"], pa.list_(pa.list_(pa.float64()))),
    })
    pq.write_table(tbl, os.path.join(d, "DL_reps", "fake_split.parquet"))
    t = ka["task_df"]
    os.makedirs(os.path.join(d, "task_dfs"), exist_ok=True)
    pq.write_table(pa.table({
        "subject_id": pa.array(t["subject_id"], pa.uint8()),
        "start_time": pa.array(ts(t["start_time_min"]), pa.timestamp("us")),
        "end_time": pa.array(ts(t["end_time_min"]), pa.timestamp("us")),
        "binary": pa.array(t["binary"]), "multi_class_int": pa.array(t["multi_class_int"], pa.int64()),
        "multi_class_cat": pa.array(t["multi_class_cat"]).dictionary_encode(),
        "regression": pa.array(t["regression"], pa.float64()),
    }), os.path.join(d, "task_dfs", "fake_task.parquet"))
    for name in ("vocabulary_config.json", "inferred_measurement_configs.json"):
        with open(os.path.join(d, name), "w") as fh:
            json.dump({}, fh)
    return ka


def _norm(v):
    """None and NaN both mean 'missing'; a None value list means all missing."""
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if v is None or (isinstance(v, float) and math.isnan(v)):
        return "nan"
    return v


def _norm_values(vals, idx):
    return [["nan"] * len(i) if v is None else _norm(v) for v, i in zip(vals, idx)]


def test_dl_reps_reader_known_answers(tmp_path):
    from eventstreamgpt_amd.data.pytorch_dataset import PytorchDataset, PytorchDatasetConfig

    ka = _write_known_frame(str(tmp_path))
    for c in ka["cases"]:
        kw = {"task_df_name": "fake_task"} if c.get("task") else {}
        pyd = PytorchDataset(PytorchDatasetConfig(save_dir=tmp_path, max_seq_len=c["max_seq_len"],
                                                  min_seq_len=c["min_seq_len"], **kw), "fake_split")
        assert len(pyd) == len(c["want"]), c["name"]
        for i, want in enumerate(c["want"]):
            st = c["starts"][i]
            got = pyd._seeded_getitem(i, seed=ka["seed"])
            end = st + c["max_seq_len"]
            for k, w in want.items():
                if k.startswith("dynamic") or k == "time_delta":
                    w = w[st:end]
                if k == "dynamic_values":
                    assert _norm_values(w, got["dynamic_indices"]) == _norm(got[k]), (c["name"], i, k)
                else:
                    assert _norm(w) == _norm(got[k]), (c["name"], i, k, w, got[k])
        if c.get("task"):
            assert pyd.tasks == sorted(ka["want_task_types"]) and pyd.task_types == ka["want_task_types"]
            assert pyd.task_vocabs["binary"] == [False, True]
            b = pyd.collate([pyd[i] for i in range(len(pyd))])
            assert b.stream_labels["binary"].dtype == torch.float32
            assert b.stream_labels["multi_class_int"].tolist() == [0, 1]
            nb = pyd.batch(np.arange(len(pyd)))
            for k in FIELDS:
                _eq(getattr(nb, k), getattr(b, k), k)
        pyd.collate([pyd._seeded_getitem(i, seed=1) for i in range(len(pyd))])  # test_get_item_should_collate


def _sample_dataset(**kw):
    from eventstreamgpt_amd.data.pytorch_dataset import PytorchDataset, PytorchDatasetConfig

    return PytorchDataset(PytorchDatasetConfig(save_dir=os.path.join(GOLDEN, "sample_dl_reps"), **kw), "tuning")


def _oracle_rows():
    import pyarrow.parquet as pq
    import collate_oracle as O

    rows = pq.read_table(os.path.join(GOLDEN, "sample_dl_reps", "DL_reps", "tuning_0.parquet")).to_pylist()
    rows = [dict(r, start_time=(r["start_time"] - datetime(1970, 1, 1)).total_seconds() / 60) for r in rows]
    return O.load_rows(rows, 2)


def test_dl_reps_sample_shard_vs_oracle():
    import collate_oracle as O

    rows, mean_log, std_log = _oracle_rows()
    pyd = _sample_dataset(max_seq_len=64, subsequence_sampling_strategy="to_end",
                          do_include_start_time_min=True, do_include_subsequence_indices=True,
                          do_include_subject_id=True)
    assert len(pyd) == len(rows) == 10
    assert math.isclose(pyd.mean_log_inter_event_time_min, mean_log, rel_tol=1e-9)
    assert math.isclose(pyd.std_log_inter_event_time_min, std_log, rel_tol=1e-9)
    items = [pyd[i] for i in range(len(pyd))]
    want = [O.getitem(r, 64, "to_end", include_start_time_min=True, include_subsequence_indices=True)
            for r in rows]
    for g, w in zip(items, want):
        for k in ("time_delta", "dynamic_indices", "dynamic_measurement_indices", "static_indices",
                  "start_idx", "end_idx"):
            assert g[k] == w[k], k
        assert _norm(g["dynamic_values"]) == _norm(w["dynamic_values"])
        assert math.isclose(g["start_time"], w["start_time"], rel_tol=1e-12)
    assert [it["subject_id"] for it in items] == [r["subject_id"] for r in rows]
    # the native windowed batch equals the oracle collate of the oracle items
    nb = pyd.batch(np.arange(len(pyd)))
    ob = O.collate(want, "right", True)
    for k in FIELDS:
        if k == "time_delta":
            torch.testing.assert_close(nb.time_delta, ob[k], rtol=0, atol=0)
        else:
            _eq(getattr(nb, k), ob[k], k)
    assert nb.start_idx.tolist() == [w["start_idx"] for w in want]
    torch.testing.assert_close(nb.start_time, torch.tensor([w["start_time"] for w in want], dtype=torch.float32))


def test_dl_reps_random_windows_and_epochs(tmp_path):
    import collate_oracle as O

    rows, _, _ = _oracle_rows()
    pyd = _sample_dataset(max_seq_len=128, do_include_subsequence_indices=True, seq_padding_side="left")
    rng = np.random.default_rng(3)
    nb = pyd.batch(np.array([3, 1, 7]), rng)
    for j, i in enumerate([3, 1, 7]):
        st, en = int(nb.start_idx[j]), int(nb.end_idx[j])
        assert 0 <= st and en - st == 128 and en <= len(rows[i]["time_delta"])
        r = dict(rows[i])
        for k in ("time_delta", "dynamic_indices", "dynamic_values", "dynamic_measurement_indices"):
            r[k] = r[k][st:en]
        ob = O.collate([O.getitem(r, 128)], "left", True)
        for k in FIELDS:
            _eq(getattr(nb, k)[j:j + 1, ..., :ob[k].shape[-1]] if k.startswith("dynamic") else
                getattr(nb, k)[j:j + 1, :ob[k].shape[1]], ob[k], k)
    # an epoch over two ranks covers every subject exactly once
    seen = []
    for rank in range(2):
        for b in pyd.batches(3, shuffle=True, seed=5, rank=rank, world_size=2):
            assert b.event_mask.shape[0] <= 3
            seen.append(b.event_mask.shape[0])
    assert sum(seen) == len(pyd)
    # train subset: size honoured (subset draw is numpy's, not polars')
    from eventstreamgpt_amd.data.pytorch_dataset import PytorchDataset, PytorchDatasetConfig

    sub = PytorchDataset(PytorchDatasetConfig(save_dir=os.path.join(GOLDEN, "sample_dl_reps"),
                                              train_subset_size=4, train_subset_seed=1), "tuning")
    assert len(sub) == 10  # only the train split is subset
    import shutil

    src = os.path.join(GOLDEN, "sample_dl_reps")
    os.makedirs(tmp_path / "DL_reps")
    shutil.copy(os.path.join(src, "DL_reps", "tuning_0.parquet"), tmp_path / "DL_reps" / "train_0.parquet")
    for name in ("vocabulary_config.json", "inferred_measurement_configs.json"):
        shutil.copy(os.path.join(src, name), tmp_path / name)
    sub = PytorchDataset(PytorchDatasetConfig(save_dir=tmp_path, train_subset_size=4, train_subset_seed=1), "train")
    assert len(sub) == 4 and set(sub.subject_ids) <= set(pyd.subject_ids)
    assert len(PytorchDataset(PytorchDatasetConfig(save_dir=tmp_path, train_subset_size=0.5), "train")) == 5
    cfg = PytorchDatasetConfig(train_subset_size=0.5)
    assert cfg.train_subset_seed is not None
    with pytest.raises(ValueError):
        PytorchDatasetConfig(seq_padding_side="middle")
    with pytest.raises(ValueError):
        PytorchDatasetConfig(train_subset_size=1.5)


def test_config_set_to_dataset_from_sample_shard():
    from eventstreamgpt_amd.transformer.config import StructuredTransformerConfig

    pyd = _sample_dataset(max_seq_len=128)
    cfg = StructuredTransformerConfig(TTE_generation_layer_type="log_normal_mixture",
                                      TTE_lognormal_generation_num_components=3)
    cfg.set_to_dataset(pyd)
    assert cfg.vocab_size == 45 and cfg.max_seq_len == 128  # vocab 45 (sample vocabulary_config)
    assert cfg.mean_log_inter_event_time_min == pyd.mean_log_inter_event_time_min
    assert "eye_color" in cfg.measurement_configs


def test_packed_batch_one_buffer_roundtrip():
    """A packed batch keeps every field in one buffer; copy_ / to() preserve values and the layout, and fields
    set after packing still travel."""
    from eventstreamgpt_amd.synthetic import CONFIGS

    b = CONFIGS["C1"].batch(0, batch_size=3)
    p = b.packed()
    flat = p.flat_buffer()
    assert flat is not None and flat.dtype == torch.uint8
    for k, v in b.as_dict().items():
        assert torch.equal(getattr(p, k), v), k
    q = CONFIGS["C1"].batch(1, batch_size=3).packed()
    q.start_time = torch.arange(3.0)
    p.start_time = torch.zeros(3)
    p.copy_(q)
    for k, v in q.as_dict().items():
        assert torch.equal(getattr(p, k), v), k
    moved = q.to("cpu")
    assert moved.flat_buffer() is not None and torch.equal(moved.start_time, q.start_time)
    p.event_mask = p.event_mask.clone()  # a reassigned field breaks the packed view -> per-field path
    assert p.flat_buffer() is None
