"""Generates tests/golden/generation_ref.pt by running the REFERENCE's generation batch updates
(``GenerativeSequenceModelSamples.append_to_batch`` / ``update_last_event_data``, model_output.py:862-1070) and
its ``strip_unused_indices`` (:108-169) on CPU in this container. Never run on the GPU box.

    python tests/golden/make_generation_golden.py

Same harness as make_golden.py (import-only stubs in ``_refstubs/``). Measurement configs are plain namespaces
with the attributes the reference reads (modality, temporality, is_dropped). The fixture holds only inputs (batch,
samples, config kwargs) and the reference's outputs.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (sets up sys.path, stubs and shims)

import torch  # noqa: E402
from EventStream.transformer.config import StructuredTransformerConfig as RefConfig  # noqa: E402
from EventStream.transformer.model_output import GenerativeSequenceModelSamples as RefSamples  # noqa: E402
from EventStream.transformer.model_output import strip_unused_indices as ref_strip  # noqa: E402

from eventstreamgpt_amd.synthetic import make_batch  # noqa: E402

MEAS = {"dept": "multi_label_classification", "labs": "multivariate_regression", "HR": "univariate_regression"}

NA_LEVELS = [[], ["event_type"], ["dept", ["labs", "categorical_only"]], [["labs", "numerical_only"], "HR"]]


def ref_config(na: bool):
    kw = dict(MG.CI_BASE if not na else MG.NA_BASE, num_hidden_layers=1, hidden_size=16, head_dim=None,
              num_attention_heads=2, seq_attention_types="global", intermediate_size=16, max_seq_len=16)
    if na:
        kw.update(measurements_per_dep_graph_level=NA_LEVELS, dep_graph_attention_types="global")
    kw.update(MG.vocab_kwargs(MG.VOCAB_SMALL))
    kw["measurement_configs"] = {m: SimpleNamespace(modality=mod, temporality="dynamic", is_dropped=False)
                                 for m, mod in MEAS.items()}
    return RefConfig(**kw)


def samples(B: int, seed: int):
    g = torch.Generator().manual_seed(seed)
    v = MG.VOCAB_SMALL["vocab_sizes_by_measurement"]
    et = torch.randint(0, v["event_type"], (B,), generator=g)
    dept = (torch.rand(B, v["dept"], generator=g) < 0.15).float()
    labs_c = (torch.rand(B, v["labs"], generator=g) < 0.2).float()
    labs_r = torch.randn(B, v["labs"], generator=g)
    hr = torch.randn(B, 1, generator=g)
    hr[torch.rand(B, generator=g) < 0.4] = float("nan")
    tte = torch.rand(B, generator=g) * 50 + 0.5
    emask = torch.ones(B, dtype=torch.bool)
    emask[-1] = False
    return dict(event_mask=emask, time_to_event=tte, classification={"event_type": et, "dept": dept, "labs": labs_c},
                regression={"labs": labs_r, "HR": hr}, regression_indices={})


def batch_dict(b):
    return {k: v.clone() for k, v in b.items() if isinstance(v, torch.Tensor)}


def dist_params(d):
    """Distribution -> its defining tensors (what our heads must reproduce)."""
    D = torch.distributions
    if d is None:
        return None
    if isinstance(d, tuple):
        return [dist_params(x) for x in d]
    if isinstance(d, D.Bernoulli):
        return {"bernoulli_logits": d.logits.detach()}
    if isinstance(d, D.Categorical):
        return {"categorical_probs": d.probs.detach()}
    if isinstance(d, D.Normal):
        return {"normal_loc": d.loc.detach(), "normal_scale": d.scale.detach()}
    if isinstance(d, D.Exponential):
        return {"exponential_rate": d.rate.detach()}
    raise TypeError(type(d))


def predictions():
    """Reference forward(batch, is_generation=True[, dep_graph_el_generation_target=t]) on the ci_small / na_small
    golden models and batches: every next-event distribution's parameters (nested_attention_model.py:47-228,
    conditionally_independent_model.py:45-161)."""
    import json

    from EventStream.data.types import PytorchBatch as RefBatch
    from EventStream.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from EventStream.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    res = {}
    for name, cls, targets in (("ci_small", CIPPTForGenerativeSequenceModeling, [None]),
                               ("na_small", NAPPTForGenerativeSequenceModeling, [None, 0, 1, 2, 3])):
        fx = torch.load(os.path.join(HERE, f"{name}.pt"), weights_only=True)
        model = cls(RefConfig(**json.loads(fx["config_kwargs"])))
        model.load_state_dict(fx["state_dict"])
        model.eval()
        per_t = {}
        for t in targets:
            kw = {"use_cache": False} if t is None else {"dep_graph_el_generation_target": t, "use_cache": False}
            with torch.no_grad():
                o = model(RefBatch(**fx["batch"]), is_generation=True, **kw)
            p = o.preds
            per_t[str(t)] = {"classification": {k: dist_params(v) for k, v in (p.classification or {}).items()},
                             "regression": {k: dist_params(v) for k, v in (p.regression or {}).items()},
                             "time_to_event": dist_params(p.time_to_event)}
        res[name] = per_t
    return res


def main():
    from EventStream.data.types import PytorchBatch as RefBatch

    out = {"meas": MEAS, "na_levels": NA_LEVELS, "cases": []}
    for case_i, (B, L, M, seed) in enumerate([(4, 6, 6, 31), (3, 5, 4, 32)]):
        b = make_batch(MG.VOCAB_SMALL, B, L, M, seed=seed, left_pad_first=True)
        b.start_time = torch.arange(B, dtype=torch.float32) * 100.0
        rb = RefBatch(**b.as_dict())
        s = samples(B, seed + 100)
        rs = RefSamples(**s)
        ci_cfg = ref_config(False)
        na_cfg = ref_config(True)

        # The reference's update_last_event_data writes into its input's tensors when no re-padding is needed, so
        # every call gets a fresh copy and every output is snapshotted before the next call.
        def fresh(d):
            return RefBatch(**{k: v.clone() for k, v in d.items()})

        appended = batch_dict(rs.append_to_batch(rb, ci_cfg))
        updated = batch_dict(rs.update_last_event_data(fresh(appended), ci_cfg))
        na1 = batch_dict(rs.update_last_event_data(fresh(appended), na_cfg, measurements_to_fill={"event_type"}))
        na2 = batch_dict(rs.update_last_event_data(fresh(na1), na_cfg,
                                                   measurements_to_fill={"dept", ("labs", "categorical_only")}))
        na3 = batch_dict(rs.update_last_event_data(fresh(na2), na_cfg,
                                                   measurements_to_fill={("labs", "numerical_only"), "HR"}))
        out["cases"].append(dict(batch=b.as_dict(), samples=s, appended=appended, updated=updated, na1=na1, na2=na2,
                                 na3=na3))
    # strip_unused_indices known answers on ragged rows (zeros interleaved, empty rows).
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, 5, (6, 9), generator=g) * (torch.rand(6, 9, generator=g) < 0.5).long()
    idx[2] = 0
    vals = torch.randn(6, 9, generator=g)
    out["strip"] = dict(idx=idx, vals=vals, want=ref_strip(idx, vals))
    out["predictions"] = predictions()
    torch.save(out, os.path.join(HERE, "generation_ref.pt"))
    print("wrote generation_ref.pt")


if __name__ == "__main__":
    main()
