"""Generates the batch-producer fixtures (collate and the DL_reps reader).

    python tests/golden/make_collate_golden.py

Two kinds of fixture, both data only:

* ``collate_known_answers.json`` / ``dl_reps_known_answers.json``: the inputs and expected outputs of the
  reference's own tests (``tests/data/test_pytorch_dataset.py``: the DL_REP_DF frame and WANT_SUBJ_* items
  ``:27-300``, ``test_get_item`` ``:402-484``, ``test_dynamic_collate_fn`` ``:486-689``, ``test_collate_fn``
  ``:691-826``), transcribed as values.
* ``collate_ref.pt``: seeded random ragged batches (empty events, None value lists, None / NaN values, NaN time deltas,
  empty static lists, left and right padding) and what the REFERENCE ``PytorchDataset.collate`` (run here, in the
  survey container, with the ``_refstubs`` import stand-ins) returned for them. Never run on the GPU box.
"""
from __future__ import annotations

import json
import math
import os
import sys
from datetime import datetime, timedelta

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
NAN = float("nan")


def known_answers():
    # test_dynamic_collate_fn (:486-531)
    s1 = {"time_delta": [0.0, 1440.0, 2880.0, 4320.0],
          "dynamic_indices": [[1, 4], [2, 7, 7, 7, 8, 8], [1, 5], [1, 4]],
          "dynamic_values": [[NAN, NAN], [NAN, 1, 2, 3, 4, 5], [NAN, NAN], [NAN, NAN]],
          "dynamic_measurement_indices": [[1, 2], [1, 3, 3, 3, 3, 3], [1, 2], [1, 2]]}
    s2 = {"time_delta": [0.0, 5, 10],
          "dynamic_indices": [[1, 4, 3], [2, 7, 7, 7], [1, 5]],
          "dynamic_values": [[NAN, NAN, NAN], [NAN, 8, 9, 10], [NAN, NAN]],
          "dynamic_measurement_indices": [[1, 2, 2], [1, 3, 3, 3], [1, 2]]}
    z6 = [0] * 6
    dyn_right = {
        "event_mask": [[1, 1, 1, 1], [1, 1, 1, 0]],
        "time_delta": [[0.0, 1440.0, 2880.0, 4320.0], [0, 5, 10, 0]],
        "dynamic_indices": [[[1, 4, 0, 0, 0, 0], [2, 7, 7, 7, 8, 8], [1, 5, 0, 0, 0, 0], [1, 4, 0, 0, 0, 0]],
                            [[1, 4, 3, 0, 0, 0], [2, 7, 7, 7, 0, 0], [1, 5, 0, 0, 0, 0], z6]],
        "dynamic_measurement_indices": [[[1, 2, 0, 0, 0, 0], [1, 3, 3, 3, 3, 3], [1, 2, 0, 0, 0, 0],
                                         [1, 2, 0, 0, 0, 0]],
                                        [[1, 2, 2, 0, 0, 0], [1, 3, 3, 3, 0, 0], [1, 2, 0, 0, 0, 0], z6]],
        "dynamic_values": [[z6, [0, 1, 2, 3, 4, 5], z6, z6], [z6, [0, 8, 9, 10, 0, 0], z6, z6]],
        "dynamic_values_mask": [[z6, [0, 1, 1, 1, 1, 1], z6, z6], [z6, [0, 1, 1, 1, 0, 0], z6, z6]],
    }
    dyn_left = {
        "event_mask": [[1, 1, 1, 1], [0, 1, 1, 1]],
        "time_delta": [[0.0, 1440.0, 2880.0, 4320.0], [0, 0, 5, 10]],
        "dynamic_indices": [dyn_right["dynamic_indices"][0],
                            [z6, [1, 4, 3, 0, 0, 0], [2, 7, 7, 7, 0, 0], [1, 5, 0, 0, 0, 0]]],
        "dynamic_measurement_indices": [dyn_right["dynamic_measurement_indices"][0],
                                        [z6, [1, 2, 2, 0, 0, 0], [1, 3, 3, 3, 0, 0], [1, 2, 0, 0, 0, 0]]],
        "dynamic_values": [dyn_right["dynamic_values"][0], [z6, z6, [0, 8, 9, 10, 0, 0], z6]],
        "dynamic_values_mask": [dyn_right["dynamic_values_mask"][0], [z6, z6, [0, 1, 1, 1, 0, 0], z6]],
    }
    # test_collate_fn (:691-826)
    ages = [[1.0, 1 + 1 / 365 + 14 / (24 * 365), 1 + 2 / 365 + 10 / (24 * 365), 1 + 3 / 365 + 23 / (24 * 365)],
            [2 + 15 / (24 * 365), 2 + 1 / 365 + 2 / (24 * 365)]]
    t1 = {"time_delta": [0.0, (24 + 14) * 60.0, (2 * 24 + 10) * 60.0, (3 * 24 + 23) * 60.0],
          "static_indices": [16], "static_measurement_indices": [6],
          "dynamic_indices": [[1, 7, 9, 11], [2, 4, 4, 4, 5, 5, 9, 12], [1, 8, 9, 13], [1, 7, 9, 14]],
          "dynamic_values": [[NAN, NAN, ages[0][0], NAN], [NAN, 1.0, 2.0, 3.0, 4.0, 5.0, ages[0][1], NAN],
                             [NAN, NAN, ages[0][2], NAN], [NAN, NAN, ages[0][3], NAN]],
          "dynamic_measurement_indices": [[1, 3, 4, 5], [1, 2, 2, 2, 2, 2, 4, 5], [1, 3, 4, 5], [1, 3, 4, 5]]}
    t2 = {"time_delta": [0.0, 11 * 60.0], "static_indices": [17], "static_measurement_indices": [6],
          "dynamic_indices": [[1, 7, 9, 12], [2, 4, 5, 9, 11]],
          "dynamic_values": [[NAN, NAN, ages[1][0], NAN], [NAN, 1.0, 5.0, ages[1][1], NAN]],
          "dynamic_measurement_indices": [[1, 3, 4, 5], [1, 2, 2, 4, 5]]}
    z8 = [0] * 8
    full = {
        "event_mask": [[1, 1, 1, 1], [1, 1, 0, 0]],
        "time_delta": [[0.0, (24 + 14) * 60.0, (2 * 24 + 10) * 60.0, (3 * 24 + 23) * 60.0], [0.0, 660.0, 0.0, 0.0]],
        "dynamic_indices": [[[1, 7, 9, 11, 0, 0, 0, 0], [2, 4, 4, 4, 5, 5, 9, 12], [1, 8, 9, 13, 0, 0, 0, 0],
                             [1, 7, 9, 14, 0, 0, 0, 0]],
                            [[1, 7, 9, 12, 0, 0, 0, 0], [2, 4, 5, 9, 11, 0, 0, 0], z8, z8]],
        "dynamic_measurement_indices": [[[1, 3, 4, 5, 0, 0, 0, 0], [1, 2, 2, 2, 2, 2, 4, 5],
                                         [1, 3, 4, 5, 0, 0, 0, 0], [1, 3, 4, 5, 0, 0, 0, 0]],
                                        [[1, 3, 4, 5, 0, 0, 0, 0], [1, 2, 2, 4, 5, 0, 0, 0], z8, z8]],
        "dynamic_values": [[[0, 0, ages[0][0], 0, 0, 0, 0, 0], [0, 1.0, 2.0, 3.0, 4.0, 5.0, ages[0][1], 0],
                            [0, 0, ages[0][2], 0, 0, 0, 0, 0], [0, 0, ages[0][3], 0, 0, 0, 0, 0]],
                           [[0, 0, ages[1][0], 0, 0, 0, 0, 0], [0, 1.0, 5.0, ages[1][1], 0, 0, 0, 0], z8, z8]],
        "dynamic_values_mask": [[[0, 0, 1, 0, 0, 0, 0, 0], [0, 1, 1, 1, 1, 1, 1, 0], [0, 0, 1, 0, 0, 0, 0, 0],
                                 [0, 0, 1, 0, 0, 0, 0, 0]],
                                [[0, 0, 1, 0, 0, 0, 0, 0], [0, 1, 1, 1, 0, 0, 0, 0], z8, z8]],
        "static_indices": [[16], [17]],
        "static_measurement_indices": [[6], [6]],
    }
    return {
        "source": "reference tests/data/test_pytorch_dataset.py:486-826",
        "cases": [
            {"name": "dynamic_right", "padding": "right", "static": False, "items": [s1, s2], "want": dyn_right},
            {"name": "dynamic_left", "padding": "left", "static": False, "items": [s1, s2], "want": dyn_left},
            {"name": "static_and_dynamic", "padding": "right", "static": True, "items": [t1, t2], "want": full},
        ],
    }


def dl_reps_known_answers():
    """DL_REP_DF and the WANT_SUBJ_* items (test_pytorch_dataset.py:27-300) with test_get_item's cases."""
    V = {"ET1": 1, "ET2": 2, "s1_UNK": 3, "foo": 4, "bar": 5, "k1": 7, "k4": 10, "sl_UNK": 11, "ur": 14, "m1": 16,
         "m2": 17, "V1": 19, "V3": 21}
    Mx = {"event_type": 1, "static1": 2, "mlc": 3, "slc": 4, "ur": 5, "mvr": 6, "static2": 7}
    starts = [datetime(1990, 1, 1), datetime(1992, 1, 1), datetime(1994, 1, 1), datetime(1991, 1, 1),
              datetime(1993, 1, 1)]
    mins = lambda ts, s: [(t - s) / timedelta(minutes=1) for t in ts]  # noqa: E731
    times = [mins([datetime(2000, 1, 1), datetime(2000, 1, 2), datetime(2000, 1, 3), datetime(2000, 2, 1)], starts[0]),
             mins([datetime(1995, 1, 1), datetime(2000, 1, 2)], starts[1]),
             mins([datetime(2001, 1, 1, 12), datetime(2001, 1, 1, 13), datetime(2001, 1, 1, 14)], starts[2]),
             None, None]
    epoch = datetime(1970, 1, 1)
    frame = {
        "subject_id": [1, 2, 3, 4, 5],
        "start_time_min": [(s - epoch) / timedelta(minutes=1) for s in starts],
        "time": times,
        "static_indices": [[V["foo"], V["V3"]], [V["V1"], V["bar"]], [], [], [V["s1_UNK"]]],
        "static_measurement_indices": [[Mx["static1"], Mx["static2"]], [Mx["static2"], Mx["static1"]], [], [],
                                       [Mx["static1"]]],
        "dynamic_indices": [
            [[V["ET1"], V["sl_UNK"], V["k1"], V["k4"]], [V["ET2"], V["ur"], V["m1"], V["m2"]], [V["ET2"], V["m1"]],
             [V["ET2"]]],
            [[V["ET2"]], [V["ET2"], V["ur"]]],
            [[V["ET1"]], [V["ET1"], V["sl_UNK"]], [V["ET1"]]],
            None, None],
        "dynamic_measurement_indices": [
            [[1, Mx["slc"], Mx["mlc"], Mx["mlc"]], [1, Mx["ur"], Mx["mvr"], Mx["mvr"]], [1, Mx["mvr"]], [1]],
            [[1], [1, Mx["ur"]]],
            [[1], [1, Mx["slc"]], [1]],
            None, None],
        "dynamic_values": [[[None, None, None, None], [None, 0.1, 0.3, 1.2], [None, NAN], [None]],
                           [[None], [None, 0.2]], [[None], [None, None], [None]], None, None],
    }
    want = []
    for i in range(3):
        t = times[i]
        want.append({
            "time_delta": [t[j + 1] - t[j] for j in range(len(t) - 1)] + [1],
            "static_indices": frame["static_indices"][i],
            "static_measurement_indices": frame["static_measurement_indices"][i],
            "dynamic_indices": frame["dynamic_indices"][i],
            "dynamic_measurement_indices": frame["dynamic_measurement_indices"][i],
            "dynamic_values": frame["dynamic_values"][i] if i < 2 else [None, None, None],
        })
    task = {"subject_id": [1, 3, 4],
            "start_time_min": [(datetime(2000, 1, 1) - epoch) / timedelta(minutes=1),
                               (datetime(2001, 1, 1, 12, 30) - epoch) / timedelta(minutes=1),
                               (datetime(1995, 1, 1) - epoch) / timedelta(minutes=1)],
            "end_time_min": [(datetime(2000, 1, 3) - epoch) / timedelta(minutes=1),
                             (datetime(2001, 1, 1, 14, 30) - epoch) / timedelta(minutes=1),
                             (datetime(2000, 1, 3) - epoch) / timedelta(minutes=1)],
            "binary": [True, False, True], "multi_class_int": [0, 1, 2], "multi_class_cat": ["a", "a", "b"],
            "regression": [1.2, 3.2, 1.5]}
    task_want = []
    for w, lab, (st, en) in zip((want[0], want[2]),
                                ({"binary": True, "multi_class_int": 0, "multi_class_cat": 0, "regression": 1.2},
                                 {"binary": False, "multi_class_int": 1, "multi_class_cat": 0, "regression": 3.2}),
                                ((0, 2), (1, 3))):
        n = en - st
        it = {k: (v[st:en] if k.startswith("dynamic") else v) for k, v in w.items()}
        it["time_delta"] = [t if i < n - 1 else 1 for i, t in enumerate(w["time_delta"][st:en])]
        task_want.append({**lab, **it})
    return {
        "source": "reference tests/data/test_pytorch_dataset.py:27-300 (frame, wants), :402-484 (test_get_item)",
        "frame": frame,
        "task_df": task,
        "want_task_types": {"binary": "binary_classification", "multi_class_int": "multi_class_classification",
                            "multi_class_cat": "multi_class_classification", "regression": "regression"},
        "cases": [
            {"name": "uncut", "max_seq_len": 4, "min_seq_len": 2, "want": want, "starts": [0, 0, 0]},
            {"name": "cut", "max_seq_len": 3, "min_seq_len": 2, "want": want, "starts": [0, 0, 0]},
            {"name": "drop_short", "max_seq_len": 4, "min_seq_len": 3, "want": [want[0], want[2]], "starts": [0, 0]},
            {"name": "task", "max_seq_len": 4, "min_seq_len": 2, "task": True, "want": task_want,
             "starts": [0, 0]},
        ],
        "seed": 1,
    }


def random_items(rng, B, L, M, S, nan_td=False):
    items = []
    for b in range(B):
        n = int(rng.integers(1, L + 1))
        it = {"time_delta": [float(x) for x in rng.exponential(30.0, n)], "dynamic_indices": [],
              "dynamic_values": [], "dynamic_measurement_indices": []}
        if nan_td and n > 1:
            it["time_delta"][int(rng.integers(0, n))] = NAN
        for _ in range(n):
            k = int(rng.integers(0, M + 1))
            it["dynamic_indices"].append([int(x) for x in rng.integers(1, 5000, k)])
            it["dynamic_measurement_indices"].append([int(x) for x in rng.integers(1, 6, k)])
            if rng.random() < 0.15:  # a whole event without values (the reader's null list)
                it["dynamic_values"].append(None)
                continue
            vals = [float(x) for x in rng.normal(0, 2, k)]
            for j in range(k):
                r = rng.random()
                if r < 0.3:
                    vals[j] = None
                elif r < 0.5:
                    vals[j] = NAN
            it["dynamic_values"].append(vals)
        s = int(rng.integers(0, S + 1))
        it["static_indices"] = [int(x) for x in rng.integers(1, 100, s)]
        it["static_measurement_indices"] = [int(x) for x in rng.integers(1, 4, s)]
        items.append(it)
    return items


def reference_collate_cases():
    import numpy as np

    np.NaN = np.nan  # the reference predates numpy 2 (its env pins numpy 1.x)
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(HERE, "_refstubs"))
    import torch
    from EventStream.data.config import SeqPaddingSide
    from EventStream.data.pytorch_dataset import PytorchDataset

    class _Cfg:
        do_include_start_time_min = False
        do_include_subsequence_indices = False
        do_include_subject_id = False

    rng = np.random.default_rng(20261016)
    cases = []
    for i, (B, L, M, S, side, static, nan_td) in enumerate([
        (4, 6, 5, 3, "right", True, False), (5, 9, 7, 2, "left", True, True), (3, 5, 4, 0, "right", False, True),
        (8, 12, 9, 4, "left", False, False), (6, 20, 16, 5, "right", True, True),
    ]):
        items = random_items(rng, B, L, M, S, nan_td)
        pyd = object.__new__(PytorchDataset)
        pyd.config = _Cfg()
        pyd.seq_padding_side = SeqPaddingSide.RIGHT if side == "right" else SeqPaddingSide.LEFT
        pyd.do_produce_static_data = static
        pyd.has_task = False
        out = pyd.collate(items)
        want = {k: v for k, v in vars(out).items() if isinstance(v, torch.Tensor)}
        cases.append({"name": f"random{i}", "padding": side, "static": static,
                      "items_json": json.dumps(items), "want": want})
    return cases


if __name__ == "__main__":
    import torch

    with open(os.path.join(HERE, "collate_known_answers.json"), "w") as f:
        json.dump(known_answers(), f)
    with open(os.path.join(HERE, "dl_reps_known_answers.json"), "w") as f:
        json.dump(dl_reps_known_answers(), f)
    torch.save(reference_collate_cases(), os.path.join(HERE, "collate_ref.pt"))
    print("wrote collate_known_answers.json, dl_reps_known_answers.json, collate_ref.pt")
