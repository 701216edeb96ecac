"""Synthetic EHR-shaped batches and the benchmark configurations C1–C5 (SURVEY.md §8 "Config restatement").

There is no network and no shipped train split, so every throughput / parity run uses batches drawn here:

* vocabulary: ``event_type`` (single-label, 8), ``dept`` (multi-label), ``labs`` (multivariate regression, which
  the reference's ETL also lists as multi-label, ``dataset_base.py:1133-1139``) and ``HR`` (univariate
  regression); offsets start at 1 (0 = padding);
* lengths L_b ~ U[0.75 L, L] with L_0 = L, right padding; elements per event ~ U[3, M]; slot 0 is the event
  type, other slots uniform over {dept, labs, HR}; values N(0,1) on labs/HR; time deltas exp(N(3,1)) minutes;
  2 static elements per subject from the event-type range (measurement index 1).

Batches are generated on the CPU from ``torch.Generator(seed)`` so they are bit-identical everywhere.
"""
from __future__ import annotations

import copy
import math
from dataclasses import dataclass, field

import torch

from .data.types import PytorchBatch

MEASUREMENTS_IDXMAP = {"event_type": 1, "dept": 2, "labs": 3, "HR": 4}


def vocabulary(n_event_types: int = 8, n_dept: int = 1000, n_labs: int = 200) -> dict:
    """A ``vocabulary_config.json``-shaped dict for the synthetic measurements."""
    sizes = {"event_type": n_event_types, "dept": n_dept, "labs": n_labs}
    offsets = {"event_type": 1}
    offsets["dept"] = offsets["event_type"] + n_event_types
    offsets["labs"] = offsets["dept"] + n_dept
    offsets["HR"] = offsets["labs"] + n_labs
    return {
        "vocab_sizes_by_measurement": sizes,
        "vocab_offsets_by_measurement": offsets,
        "measurements_idxmap": dict(MEASUREMENTS_IDXMAP),
        "measurements_per_generative_mode": {
            "single_label_classification": ["event_type"],
            "multi_label_classification": ["dept", "labs"],
            "multivariate_regression": ["labs"],
            "univariate_regression": ["HR"],
        },
        "event_types_idxmap": {f"type_{i}": i + 1 for i in range(n_event_types)},
    }


@dataclass
class BenchConfig:
    """One of the configurations C1–C5."""

    cfg_id: int
    name: str
    batch_size: int
    seq_len: int
    n_elements: int
    vocab: dict
    model_kwargs: dict = field(default_factory=dict)
    n_static: int = 2

    def model_config(self, **overrides):
        from .transformer.config import StructuredTransformerConfig

        kw = copy.deepcopy(self.model_kwargs)
        kw.update(overrides)
        cfg = StructuredTransformerConfig(**kw)
        cfg.set_to_vocabulary(self.vocab, max_seq_len=self.seq_len)
        if cfg.TTE_generation_layer_type == "log_normal_mixture":
            # time_delta = exp(N(3,1)) minutes  =>  (mean_log, std_log) = (3, 1): exercises the affine path.
            cfg.mean_log_inter_event_time_min = 3.0
            cfg.std_log_inter_event_time_min = 1.0
        return cfg

    def batch(self, step: int = 0, batch_size: int | None = None, device="cpu") -> PytorchBatch:
        return make_batch(
            self.vocab, batch_size or self.batch_size, self.seq_len, self.n_elements,
            seed=1000 * self.cfg_id + step, n_static=self.n_static, device=device,
        )


_CI = dict(structured_event_processing_mode="conditionally_independent", do_full_block_in_seq_attention=None,
           do_full_block_in_dep_graph_attention=None, dep_graph_window_size=None)


def _ci(**kw):
    d = dict(_CI)
    d.update(kw)
    return d


CONFIGS: dict[str, BenchConfig] = {
    "C1": BenchConfig(1, "CI tiny 2L d=64", 32, 256, 16, vocabulary(8, 39, 20),
                      _ci(num_hidden_layers=2, hidden_size=64, head_dim=None, num_attention_heads=4,
                          seq_attention_types=["local", "global"], seq_window_size=32, intermediate_size=32)),
    "C2": BenchConfig(2, "CI 6L d=256 global", 32, 256, 16, vocabulary(8, 1000, 200),
                      _ci(num_hidden_layers=6, hidden_size=256, head_dim=None, num_attention_heads=4,
                          seq_attention_types="global", intermediate_size=1024)),
    "C3": BenchConfig(3, "CI 12L d=512 global/local-32", 32, 512, 16, vocabulary(8, 1000, 200),
                      _ci(num_hidden_layers=12, hidden_size=512, head_dim=None, num_attention_heads=8,
                          seq_attention_types=["global", "local"], seq_window_size=32, intermediate_size=2048)),
    "C4": BenchConfig(4, "NA 6L d=256 G=4 split", 32, 256, 16, vocabulary(8, 1000, 200),
                      dict(structured_event_processing_mode="nested_attention", num_hidden_layers=6,
                           hidden_size=256, head_dim=None, num_attention_heads=4, seq_attention_types="global",
                           dep_graph_attention_types="global", dep_graph_window_size=None,
                           intermediate_size=1024, do_full_block_in_seq_attention=True,
                           do_full_block_in_dep_graph_attention=True, do_split_embeddings=True,
                           categorical_embedding_dim=64, numerical_embedding_dim=64,
                           measurements_per_dep_graph_level=[
                               [], ["event_type"], ["dept", ("labs", "categorical_only")],
                               [("labs", "numerical_only"), "HR"]])),
    "C5": BenchConfig(5, "CI L=1024 LNM K=8 10k vocab", 16, 1024, 32, vocabulary(8, 10000, 200),
                      _ci(num_hidden_layers=6, hidden_size=256, head_dim=None, num_attention_heads=4,
                          seq_attention_types="global", intermediate_size=1024,
                          TTE_generation_layer_type="log_normal_mixture",
                          TTE_lognormal_generation_num_components=8)),
}


def make_batch(vocab: dict, batch_size: int, seq_len: int, n_elements: int, seed: int, n_static: int = 2,
               device="cpu", left_pad_first: bool = False) -> PytorchBatch:
    """Draws one synthetic ``PytorchBatch`` (see module docstring). Deterministic in ``seed``."""
    g = torch.Generator().manual_seed(seed)
    B, L, M = batch_size, seq_len, n_elements
    sizes = vocab["vocab_sizes_by_measurement"]
    offs = vocab["vocab_offsets_by_measurement"]
    midx = vocab["measurements_idxmap"]

    lo = max(1, int(math.ceil(0.75 * L)))
    lengths = torch.randint(lo, L + 1, (B,), generator=g)
    lengths[0] = L
    pos = torch.arange(L)
    event_mask = pos[None, :] < lengths[:, None]
    if left_pad_first and B > 1:
        # Subject 1 left-padded (generation-style padding; the reference's invariance tests use one).
        event_mask[1] = pos >= (L - lengths[1])

    n_el = torch.randint(3, M + 1, (B, L), generator=g)
    slot = torch.arange(M)
    present = (slot[None, None, :] < n_el[..., None]) & event_mask[..., None]

    # Measurement per slot: slot 0 event_type; others uniform over dept / labs / HR.
    other = torch.randint(0, 3, (B, L, M), generator=g)
    meas_choices = torch.tensor([midx["dept"], midx["labs"], midx["HR"]])
    meas = meas_choices[other]
    meas[..., 0] = midx["event_type"]
    meas = torch.where(present, meas, torch.zeros_like(meas))

    u = torch.rand((B, L, M), generator=g, dtype=torch.float64)
    idx = torch.zeros((B, L, M), dtype=torch.long)
    for name in ("event_type", "dept", "labs"):
        sel = meas == midx[name]
        draw = offs[name] + (u * sizes[name]).floor().long().clamp_max(sizes[name] - 1)
        idx = torch.where(sel, draw, idx)
    idx = torch.where(meas == midx["HR"], torch.full_like(idx, offs["HR"]), idx)

    vals = torch.randn((B, L, M), generator=g)
    vmask = (meas == midx["labs"]) | (meas == midx["HR"])
    vals = torch.where(vmask, vals, torch.zeros_like(vals))

    td = torch.exp(3.0 + torch.randn((B, L), generator=g))
    td = torch.where(event_mask, td, torch.zeros_like(td))

    s_idx = offs["event_type"] + torch.randint(0, sizes["event_type"], (B, n_static), generator=g)
    s_meas = torch.full((B, n_static), midx["event_type"], dtype=torch.long)

    batch = PytorchBatch(
        event_mask=event_mask,
        time_delta=td.float(),
        static_indices=s_idx,
        static_measurement_indices=s_meas,
        dynamic_indices=idx,
        dynamic_measurement_indices=meas,
        dynamic_values=vals.float(),
        dynamic_values_mask=vmask,
    )
    return batch.to(device) if str(device) != "cpu" else batch
