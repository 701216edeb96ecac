"""Batch-producer throughput: native collate (+ pinned H2D when a GPU is present) vs the reference algorithm.

    python tools/producer_bench.py [--config C2] [--batches 20] [--ref-batches 2] [--out profiles/x.json]

The workload is the bench config's synthetic batches (``eventstreamgpt_amd.synthetic``) un-padded into one flat
store of subjects; each measured batch draws B subjects and collates windows of at most L events. The reference
leg runs the oracle restatement of ``PytorchDataset.collate`` (``oracle/collate_oracle.py``: per-event tensor
construction and padding, as ``pytorch_dataset.py:568-683``) on the same subjects as item dicts, on one core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from eventstreamgpt_amd.data.collate import RaggedEvents, collate_ragged  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402


def store_from_batches(cfg, n_batches: int) -> RaggedEvents:
    """Right-padded synthetic batches -> one flat store (subjects = rows of every batch)."""
    td, el_len, idx, meas, vals, ev_count, st_i, st_m = [], [], [], [], [], [], [], []
    for s in range(n_batches):
        b = cfg.batch(s)
        em = b.event_mask.numpy()
        n_ev = em.sum(1)
        present = b.dynamic_indices.numpy() != 0
        for r in range(em.shape[0]):
            n = int(n_ev[r])
            ev_count.append(n)
            td.append(b.time_delta[r, :n].double().numpy())
            p = present[r, :n]
            el_len.append(p.sum(1))
            idx.append(b.dynamic_indices[r, :n].numpy()[p])
            meas.append(b.dynamic_measurement_indices[r, :n].numpy()[p])
            v = b.dynamic_values[r, :n].double().numpy().copy()
            v[~b.dynamic_values_mask[r, :n].numpy()] = np.nan
            vals.append(v[p])
            st_i.append(b.static_indices[r].numpy())
            st_m.append(b.static_measurement_indices[r].numpy())
    ev_count = np.asarray(ev_count)
    st_count = np.array([len(x) for x in st_i])
    return RaggedEvents(
        np.concatenate([[0], np.cumsum(ev_count)[:-1]]), ev_count, np.concatenate(td),
        np.concatenate([[0], np.cumsum(np.concatenate(el_len))]), np.concatenate(idx), np.concatenate(meas),
        np.concatenate(vals), np.concatenate([[0], np.cumsum(st_count)[:-1]]), st_count, np.concatenate(st_i),
        np.concatenate(st_m))


def items_of(r: RaggedEvents, subjects) -> list[dict]:
    out = []
    for s in subjects:
        a, n = int(r.ev_start[s]), int(r.ev_count[s])
        off = r.el_off[a:a + n + 1]
        cuts = (off[1:-1] - off[0]).tolist()
        e0, e1 = int(off[0]), int(off[-1])
        s0, sc = int(r.st_start[s]), int(r.st_count[s])
        out.append({
            "time_delta": r.time_delta[a:a + n].tolist(),
            "dynamic_indices": [x.tolist() for x in np.split(r.idx[e0:e1], cuts)],
            "dynamic_measurement_indices": [x.tolist() for x in np.split(r.meas[e0:e1], cuts)],
            "dynamic_values": [[None if np.isnan(v) else v for v in x.tolist()] for x in np.split(r.vals[e0:e1], cuts)],
            "static_indices": r.st_idx[s0:s0 + sc].tolist(),
            "static_measurement_indices": r.st_meas[s0:s0 + sc].tolist(),
        })
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--ref-batches", type=int, default=2)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    B = cfg.batch_size
    store = store_from_batches(cfg, 8)
    rng = np.random.default_rng(0)
    picks = [rng.choice(store.n_subjects, B, replace=False) for _ in range(a.batches)]
    gpu = torch.cuda.is_available()
    pin = gpu
    th = a.threads or None

    def native(sel):
        b = collate_ragged(store.window(sel), "right", True, pin_memory=pin, n_threads=th)
        if gpu:
            b = b.to("cuda", non_blocking=True)
        return b

    native(picks[0])
    if gpu:
        torch.cuda.synchronize()
    events = 0
    t0 = time.perf_counter()
    for sel in picks:
        b = native(sel)
        events += int(store.ev_count[sel].sum())
    if gpu:
        torch.cuda.synchronize()
    t_nat = (time.perf_counter() - t0) / a.batches
    ev_per_batch = events / a.batches

    import oracle.collate_oracle as O

    ref_items = [items_of(store, sel) for sel in picks[:a.ref_batches]]
    t0 = time.perf_counter()
    for items in ref_items:
        O.collate(items, "right", True)
    t_ref = (time.perf_counter() - t0) / a.ref_batches
    res = {
        "workload": f"{a.config}: B={B}, L<={cfg.seq_len}, M<={cfg.n_elements}, {ev_per_batch:.0f} events/batch",
        "native_ms_per_batch": t_nat * 1e3,
        "native_events_per_s": ev_per_batch / t_nat,
        "native_includes_h2d": gpu,
        "native_threads": th or "auto",
        "reference_algorithm_ms_per_batch": t_ref * 1e3,
        "reference_algorithm_events_per_s": ev_per_batch / t_ref,
        "speedup": t_ref / t_nat,
    }
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
