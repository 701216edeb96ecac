"""Generates the golden fixtures in tests/golden/ by running the REFERENCE (Jwoo5/EventStreamGPT, read-only at
/root/reference) on CPU in the survey/oracle container. Never run on the GPU box (the reference does not travel).

    python tests/golden/make_golden.py            # writes tests/golden/*.pt and known_answers.json

Harness: ``_refstubs/`` holds import-only stand-ins for packages the container lacks (polars, hydra, omegaconf,
ml-mixins, sparklines, lightning) plus a restatement of ``pytorch_lognormal_mixture`` (third party, pinned
0.0.1 in the reference's env.yml:409, not installable here). ``PreTrainedModel.get_head_mask`` (removed in
transformers 5.x; the reference pins 4.27.4) is shimmed. No reference source is copied: each fixture holds only
inputs (config kwargs, weights, batch) and the reference's outputs (losses, encodings, gradients).

Batches come from the product's own generator (``eventstreamgpt_amd.synthetic.make_batch``), seeded.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(HERE, "_refstubs"))

import torch  # noqa: E402
from transformers.modeling_utils import PreTrainedModel  # noqa: E402

PreTrainedModel.get_head_mask = (  # noqa: E731
    lambda self, hm, n, is_attention_chunked=False: [None] * n if hm is None else hm
)

from EventStream.data.types import PytorchBatch as RefBatch  # noqa: E402
from EventStream.transformer.conditionally_independent_model import (  # noqa: E402
    CIPPTForGenerativeSequenceModeling,
)
from EventStream.transformer.config import StructuredTransformerConfig as RefConfig  # noqa: E402
from EventStream.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling  # noqa: E402

from eventstreamgpt_amd.synthetic import make_batch, vocabulary  # noqa: E402

torch.set_num_threads(8)

VOCAB_SMALL = vocabulary(8, 39, 20)  # V = 69 (C1's synthetic vocabulary)


def vocab_kwargs(v):
    sizes = v["vocab_sizes_by_measurement"]
    offs = v["vocab_offsets_by_measurement"]
    total = sum(sizes.values()) + min(offs.values()) + (len(offs) - len(sizes))
    mpg = dict(v["measurements_per_generative_mode"])
    return dict(
        vocab_sizes_by_measurement=dict(sizes, HR=1),
        vocab_offsets_by_measurement=dict(offs),
        measurements_idxmap=dict(v["measurements_idxmap"]),
        measurements_per_generative_mode=mpg,
        vocab_size=total,
    )


CI_BASE = dict(structured_event_processing_mode="conditionally_independent", do_full_block_in_seq_attention=None,
               do_full_block_in_dep_graph_attention=None, dep_graph_window_size=None,
               attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
NA_BASE = dict(structured_event_processing_mode="nested_attention",
               attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)

CASES = {
    # C1-like: JOINT, static SUM_ALL, [local(w=4), global], exponential TTE, right padding.
    "ci_small": dict(
        model=dict(CI_BASE, num_hidden_layers=2, hidden_size=32, head_dim=None, num_attention_heads=2,
                   seq_attention_types=["local", "global"], seq_window_size=4, intermediate_size=64,
                   max_seq_len=32),
        batch=dict(B=4, L=32, M=8, seed=11, left_pad=False)),
    # JOINT + measurement-index normalisation + LogNormalMixture (affine path mean_log=3, std_log=1), left pad.
    "ci_lnm_norm": dict(
        model=dict(CI_BASE, num_hidden_layers=2, hidden_size=32, head_dim=None, num_attention_heads=2,
                   seq_attention_types="global", intermediate_size=64, max_seq_len=24,
                   do_normalize_by_measurement_index=True, TTE_generation_layer_type="log_normal_mixture",
                   TTE_lognormal_generation_num_components=4, mean_log_inter_event_time_min=3.0,
                   std_log_inter_event_time_min=1.0, static_embedding_weight=0.3, dynamic_embedding_weight=0.6),
        batch=dict(B=4, L=24, M=8, seed=12, left_pad=True)),
    # SPLIT embeddings + normalisation, static SUM_ALL, head_dim 32 x 2 heads, local window 3, gelu_new.
    "ci_split": dict(
        model=dict(CI_BASE, num_hidden_layers=2, hidden_size=64, head_dim=None, num_attention_heads=2,
                   seq_attention_types=["global", "local"], seq_window_size=3, intermediate_size=128,
                   max_seq_len=16, do_split_embeddings=True, categorical_embedding_dim=24,
                   numerical_embedding_dim=16, do_normalize_by_measurement_index=True,
                   categorical_embedding_weight=0.7, numerical_embedding_weight=0.2),
        batch=dict(B=3, L=16, M=8, seed=13, left_pad=False)),
    # NA, SPLIT, G = 4 levels as C4, full blocks in both modules.
    "na_small": dict(
        model=dict(NA_BASE, num_hidden_layers=2, hidden_size=32, head_dim=None, num_attention_heads=2,
                   seq_attention_types="global", dep_graph_attention_types="global", dep_graph_window_size=None,
                   intermediate_size=64, max_seq_len=16, do_full_block_in_seq_attention=True,
                   do_full_block_in_dep_graph_attention=True, do_split_embeddings=True,
                   categorical_embedding_dim=16, numerical_embedding_dim=16,
                   measurements_per_dep_graph_level=[[], ["event_type"], ["dept", ["labs", "categorical_only"]],
                                                     [["labs", "numerical_only"], "HR"]]),
        batch=dict(B=3, L=16, M=8, seed=14, left_pad=False)),
    # NA, JOINT (bucket leak), attention-only modules (no residual), local dep-graph window 2, left pad.
    "na_joint_attn": dict(
        model=dict(NA_BASE, num_hidden_layers=2, hidden_size=32, head_dim=None, num_attention_heads=4,
                   seq_attention_types=["local", "global"], seq_window_size=5,
                   dep_graph_attention_types=["local"], dep_graph_window_size=2,
                   intermediate_size=48, max_seq_len=16, do_full_block_in_seq_attention=False,
                   do_full_block_in_dep_graph_attention=False,
                   measurements_per_dep_graph_level=[[], ["event_type"], ["dept", "labs", "HR"]]),
        batch=dict(B=3, L=16, M=8, seed=15, left_pad=True)),
}


def to_ref_batch(b) -> RefBatch:
    return RefBatch(**{k: v for k, v in b.as_dict().items()})


def run_case(name, spec):
    torch.manual_seed(0)
    kw = dict(spec["model"])
    kw.update(vocab_kwargs(VOCAB_SMALL))
    cfg = RefConfig(**kw)
    model_cls = (CIPPTForGenerativeSequenceModeling if kw["structured_event_processing_mode"] ==
                 "conditionally_independent" else NAPPTForGenerativeSequenceModeling)
    model = model_cls(cfg)
    model.train()
    bs = spec["batch"]
    b = make_batch(VOCAB_SMALL, bs["B"], bs["L"], bs["M"], seed=bs["seed"], left_pad_first=bs["left_pad"])
    rb = to_ref_batch(b)

    captured = {}
    h = model.encoder.input_layer.register_forward_hook(lambda m, i, o: captured.__setitem__("input_embeds", o))
    out = model(rb)
    h.remove()
    enc = model.encoder(rb).last_hidden_state
    out.loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    fx = {
        "config_kwargs": json.dumps(kw),
        "state_dict": {k: v.detach().clone() for k, v in model.state_dict().items()},
        "batch": b.as_dict(),
        "loss": out.loss.detach(),
        "classification": {k: v.detach() for k, v in out.losses.classification.items()},
        "regression": {k: v.detach() for k, v in out.losses.regression.items()},
        "tte_nll": out.losses.time_to_event.detach(),
        "input_embeds": captured["input_embeds"].detach(),
        "encoded": enc.detach(),
        "grads": grads,
    }
    path = os.path.join(HERE, f"{name}.pt")
    torch.save(fx, path)
    print(f"{name}: loss={out.loss.item():.6f} -> {path} ({os.path.getsize(path) // 1024} KiB)")


def known_answers():
    """Scalar known answers of the reference's own tests, re-derived by running its code here."""
    from EventStream.transformer.generative_layers import LogNormalMixtureTTELayer
    from EventStream.transformer.utils import safe_weighted_avg, weighted_loss
    from EventStream.data.data_embedding_layer import DataEmbeddingLayer

    ka = {}
    ka["weighted_loss"] = weighted_loss(torch.FloatTensor([[1, 2, 3], [4, 5, 6]]),
                                        torch.FloatTensor([[1, 1, 1], [1, 0, 0]])).item()
    X = torch.FloatTensor([[1, 2, 3], [4, 5, 6]])
    ka["safe_weighted_avg"] = [t.tolist() for t in safe_weighted_avg(X, X.clone())]
    ka["meas_norm"] = DataEmbeddingLayer.get_measurement_index_normalziation(
        torch.LongTensor([[1, 2, 5, 2, 2], [1, 3, 5, 3, 0]])).tolist()
    torch.manual_seed(1)
    lay = LogNormalMixtureTTELayer(in_dim=4, num_components=3, mean_log_inter_time=2.0, std_log_inter_time=0.5)
    T = torch.randn(2, 5, 4)
    x = torch.rand(2, 5) * 10 + 0.1
    d = lay(T)
    ka["lnm_affine"] = {"weight": lay.proj.weight.tolist(), "bias": lay.proj.bias.tolist(), "T": T.tolist(),
                        "x": x.tolist(), "log_prob": d.log_prob(x).tolist(), "mean": d.mean.tolist()}
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(ka, f, indent=1)
    print("known_answers.json written")


if __name__ == "__main__":
    for n, s in CASES.items():
        run_case(n, s)
    known_answers()
