"""The HIP input layer (torch.ops.esgpt.embed_joint / embed_split_bags) against the reference's own
DataEmbeddingLayer known answers (tests/data/test_data_embedding_layer.py:255-346 JOINT, :348-576 SPLIT,
:732-913 full forward with static DROP / SUM_ALL; identity tables, fixture transcribed by
tests/golden/make_embedding_known_answers.py).

The gather is bit-exact: every answer whose values are exact in f32 (all but two of them) must come out
``torch.equal``; the two SUM_ALL cases with weights 1/3, 2/3 are compared at one f32 ulp. The reference's bags are
[N, M] rows; here each row is one event of a one-subject batch (event mask all True), which is how the layer sees
them in the model. The SPLIT ``cat_mask`` case has a per-element categorical mask that no measurement-index bucket
can express (element (0, 0) and (0, 2) share measurement 1 but differ), so it is pinned through the oracle only
(tests/test_oracle_golden.py)."""
import json
import os
from fractions import Fraction

import pytest
import torch

from eventstreamgpt_amd.data.data_embedding_layer import DataEmbeddingLayer
from eventstreamgpt_amd.data.types import PytorchBatch

pytestmark = pytest.mark.gpu
DEV = "cuda"
FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "embedding_known_answers.json")))


def _t(x):
    return torch.tensor(x["data"], dtype=getattr(torch, x["dtype"]))


def _exact_in_f32(want: torch.Tensor) -> bool:
    return all(Fraction(float(v)).limit_denominator(1 << 20).denominator & (
        Fraction(float(v)).limit_denominator(1 << 20).denominator - 1) == 0 for v in want.flatten().tolist())


def _layer(c):
    prm = dict(c["params"])
    L = DataEmbeddingLayer(**prm).to(DEV)
    with torch.no_grad():
        if L.embedding_mode == "joint":
            L.embed_layer.weight.copy_(torch.eye(4))
        else:
            L.categorical_embed_layer.weight.copy_(torch.eye(4))
            L.cat_proj.weight.copy_(0.5 * torch.eye(4))
            L.cat_proj.bias.zero_()
            L.numerical_embed_layer.weight.copy_(2 * torch.eye(4))
            L.num_proj.weight.copy_(-torch.eye(4))
            L.num_proj.bias.zero_()
    return L


@pytest.mark.parametrize("case", FX["cases"], ids=[f"{c['kind']}-{i}" for i, c in enumerate(FX["cases"])])
def test_hip_input_layer_reproduces_reference_known_answers(case):
    if "cat_mask" in case and not all(all(r) for r in case["cat_mask"]["data"]):
        pytest.skip("per-element cat_mask: not expressible by measurement buckets (oracle-pinned instead)")
    want = _t(case["want"])
    L = _layer(case)
    if case["kind"] == "forward":
        batch = PytorchBatch(**{k: _t(v) for k, v in case["batch"]["PytorchBatch"].items()}).to(DEV)
        got = L(batch)
    else:
        idx = _t(case["indices"])
        N, M = idx.shape
        batch = PytorchBatch(event_mask=torch.ones(1, N, dtype=torch.bool), time_delta=torch.zeros(1, N),
                             dynamic_indices=idx[None], dynamic_measurement_indices=_t(case["measurement_indices"])[None],
                             dynamic_values=_t(case["values"])[None],
                             dynamic_values_mask=_t(case["values_mask"])[None]).to(DEV)
        got = L(batch)[0]
    got = got.detach().cpu()
    assert got.shape == want.shape
    if _exact_in_f32(want):
        assert torch.equal(got, want), (case["msg"], got, want)
    else:
        torch.testing.assert_close(got, want, rtol=1.2e-7, atol=0.0, msg=case["msg"])
