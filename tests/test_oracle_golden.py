"""The oracle (CPU restatement) against golden vectors produced by the reference itself."""
import json
import os

import pytest
import torch

import esgpt_oracle as O
from helpers import CASES, GOLDEN, load_case, rel_err


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference(name):
    fx, cfg, batch = load_case(name)
    params = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in fx["state_dict"].items()}
    out = O.model_losses(params, cfg, batch)
    assert rel_err(out["encoded"].detach(), fx["encoded"]) < 1e-5
    assert abs(out["loss"].item() - fx["loss"].item()) <= 1e-5 * abs(fx["loss"].item())
    for k, v in fx["classification"].items():
        assert abs(out["classification"][k].item() - v.item()) <= 1e-5 * max(1.0, abs(v.item()))
    for k, v in fx["regression"].items():
        assert abs(out["regression"][k].item() - v.item()) <= 1e-5 * max(1.0, abs(v.item()))
    assert abs(-out["tte_ll"].item() - fx["tte_nll"].item()) <= 1e-5 * max(1.0, abs(fx["tte_nll"].item()))
    out["loss"].backward()
    for k, g in fx["grads"].items():
        assert params[k].grad is not None, k
        assert rel_err(params[k].grad, g) < 1e-4, (k, rel_err(params[k].grad, g))


def test_known_answers():
    ka = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    assert O.weighted_loss(torch.FloatTensor([[1, 2, 3], [4, 5, 6]]),
                           torch.FloatTensor([[1, 1, 1], [1, 0, 0]])).item() == pytest.approx(ka["weighted_loss"])
    X = torch.FloatTensor([[1, 2, 3], [4, 5, 6]])
    got = O.safe_weighted_avg(X, X.clone())
    for a, b in zip(got, ka["safe_weighted_avg"]):
        torch.testing.assert_close(a, torch.tensor(b))
    torch.testing.assert_close(O.meas_index_normalization(torch.LongTensor([[1, 2, 5, 2, 2], [1, 3, 5, 3, 0]])),
                               torch.tensor(ka["meas_norm"]))
    lnm = ka["lnm_affine"]
    z = torch.nn.functional.linear(torch.tensor(lnm["T"]), torch.tensor(lnm["weight"]), torch.tensor(lnm["bias"]))
    lp = O.lnm_log_prob(z, torch.tensor(lnm["x"]), 2.0, 0.5)
    torch.testing.assert_close(lp, torch.tensor(lnm["log_prob"]), rtol=1e-5, atol=1e-5)


def test_tte_reference_known_answers():
    """Restated known answers of the reference (tests/transformer/test_model_output.py:1417-1535): batch of one
    subject with 3 events, time_delta [2, 3, 1]; parameters chosen so that
    Exponential rates are [1, 2, 3] -> LL -3.6534264097200273, and LNM (K = 2, mean_log 0, std_log 1) with
    per-position params = rows [[0..5], [1,3,..,11], [2,4,..,12]] interleaved (loc, log_scale, log_weight)
    -> LL -7.6554941334115565."""
    enc = torch.tensor([[[0.0, 1, 2, 3, 4, 5], [1, 3, 5, 7, 9, 11], [2, 4, 6, 8, 10, 12]]])
    batch = {"event_mask": torch.ones(1, 3, dtype=torch.bool), "time_delta": torch.tensor([[2.0, 3.0, 1.0]])}

    class C:
        TTE_generation_layer_type = "log_normal_mixture"
        mean_log_inter_event_time_min = 0.0
        std_log_inter_event_time_min = 1.0

    p = {"TTE_layer.proj.weight": torch.eye(6), "TTE_layer.proj.bias": torch.zeros(6)}
    ll = O.tte_log_likelihood(p, "", C, batch, enc)
    assert ll.item() == pytest.approx(-7.6554941334115565, abs=1e-5)

    C.TTE_generation_layer_type = "exponential"
    # proj picks a value whose elu+1 gives rates [1, 2, 3]: z = [0, 1, 2] = column 0 of enc.
    w = torch.zeros(1, 6)
    w[0, 0] = 1.0
    p = {"TTE_layer.proj.weight": w, "TTE_layer.proj.bias": torch.zeros(1)}
    ll = O.tte_log_likelihood(p, "", C, batch, enc)
    assert ll.item() == pytest.approx(-3.6534264097200273, abs=1e-5)


def _ka_tensor(x):
    return torch.tensor(x["data"], dtype=getattr(torch, x["dtype"]))


def test_oracle_embedding_known_answers():
    """The oracle's DataEmbeddingLayer restatement reproduces the reference's own known answers
    (tests/data/test_data_embedding_layer.py:255-346, 348-576, 732-913; fixture transcribed by
    tests/golden/make_embedding_known_answers.py)."""
    import json

    fx = json.load(open(os.path.join(GOLDEN, "embedding_known_answers.json")))
    assert len(fx["cases"]) == 9
    for c in fx["cases"]:
        prm = c["params"]
        ew = dict(mode="split" if prm.get("categorical_embedding_dim") else "joint",
                  do_normalize_by_measurement_index=prm.get("do_normalize_by_measurement_index", False),
                  static_embedding_mode=prm["static_embedding_mode"], static_weight=prm.get("static_weight", 0.5),
                  dynamic_weight=prm.get("dynamic_weight", 0.5), categorical_weight=prm.get("categorical_weight", 0.5),
                  numerical_weight=prm.get("numerical_weight", 0.5))
        p = {"e.embed_layer.weight": torch.eye(4), "e.categorical_embed_layer.weight": torch.eye(4),
             "e.cat_proj.weight": 0.5 * torch.eye(4), "e.cat_proj.bias": torch.zeros(4),
             "e.numerical_embed_layer.weight": 2 * torch.eye(4), "e.num_proj.weight": -torch.eye(4),
             "e.num_proj.bias": torch.zeros(4)}
        want = _ka_tensor(c["want"])
        if c["kind"] == "forward":
            batch = {k: _ka_tensor(v) for k, v in c["batch"]["PytorchBatch"].items()}
            got = O.data_embedding(p, "e.", ew, batch)
        else:
            got = O.embed_bags(p, "e.", ew, _ka_tensor(c["indices"]), _ka_tensor(c["measurement_indices"]),
                               _ka_tensor(c["values"]), _ka_tensor(c["values_mask"]),
                               _ka_tensor(c["cat_mask"]) if "cat_mask" in c else None)
        torch.testing.assert_close(got, want, msg=c["msg"])
