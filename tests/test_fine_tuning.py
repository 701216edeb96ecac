"""Fine-tuning head (ESTForStreamClassification) against the reference tests' known answers
(tests/golden/fine_tuning_known_answers.json; the encoder is mocked exactly as the reference test does), plus the
pooling rules on masked batches. CPU: pooling, the logit layer and the loss are host-side torch ops."""
import json
import os

import pytest
import torch

from eventstreamgpt_amd.data.types import PytorchBatch
from eventstreamgpt_amd.transformer.config import StructuredTransformerConfig
from eventstreamgpt_amd.transformer.fine_tuning_model import POOLING, ESTForStreamClassification

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "fine_tuning_known_answers.json")))


class _Hidden:
    def __init__(self, h):
        self.last_hidden_state = h


class _MockEncoder(torch.nn.Module):
    def __init__(self, h):
        super().__init__()
        self.h = h

    def forward(self, *args, **kwargs):
        return _Hidden(self.h)


@pytest.mark.parametrize("case", FX["cases"], ids=[c["msg"] for c in FX["cases"]])
def test_known_answers(case):
    kw = {**FX["default_config"], **case["config"]}
    if "id2label" in kw:
        # transformers >= 5 validates id2label as dict[int, str]: the reference's {0: False, 1: True} as strings
        kw["id2label"] = {int(k): str(v) for k, v in kw["id2label"].items()}
        kw["label2id"] = dict(kw["label2id"])
    cfg = StructuredTransformerConfig(**kw)
    m = ESTForStreamClassification(cfg)
    m.encoder = _MockEncoder(torch.tensor(case["hidden"]))
    m.logit_layer.weight = torch.nn.Parameter(torch.tensor(case["weight"]))
    m.logit_layer.bias = torch.nn.Parameter(torch.tensor(case["bias"]))
    labels = torch.tensor(case["labels"], dtype=torch.float32 if case["labels_dtype"] == "float" else torch.long)
    em = None if case["event_mask"] is None else torch.tensor(case["event_mask"])
    out = m(PytorchBatch(event_mask=em, stream_labels={"test": labels}))
    assert torch.equal(out.labels, labels)
    assert torch.allclose(out.preds, torch.tensor(case["want_preds"]))
    assert out.loss.item() == pytest.approx(case["want_loss"], rel=1e-6)


def test_masked_pooling_matches_safe_reductions():
    """max / mean pooling over valid events only, zero for a subject without events (utils.py:61-207)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 5, 4, generator=g)
    em = torch.tensor([[1, 1, 0, 1, 0], [0, 0, 0, 0, 0], [1, 1, 1, 1, 1]], dtype=torch.bool)
    b = PytorchBatch(event_mask=em)
    mx, mean = POOLING["max"](x, b), POOLING["mean"](x, b)
    for i in range(3):
        v = x[i][em[i]]
        want_max = v.max(0).values if len(v) else torch.zeros(4)
        want_mean = v.mean(0) if len(v) else torch.zeros(4)
        assert torch.allclose(mx[i], want_max) and torch.allclose(mean[i], want_mean, atol=1e-6)
    assert torch.equal(POOLING["cls"](x, b), x[:, 0]) and torch.equal(POOLING["last"](x, b), x[:, -1])
    with pytest.raises(ValueError, match="not a supported pooling method"):
        cfg = StructuredTransformerConfig(**{**FX["default_config"], "task_specific_params": {"pooling_method": "sum"}})
        m = ESTForStreamClassification(cfg)
        m.encoder = _MockEncoder(x.unsqueeze(2))
        m(PytorchBatch(event_mask=em, stream_labels={"test": torch.zeros(3, dtype=torch.long)}))


def test_oracle_restatement_known_answers():
    """The oracle's stream_classification_loss reproduces the reference's known answers (mocked encoder)."""
    import esgpt_oracle as O

    for case in FX["cases"]:
        cfg = StructuredTransformerConfig(**{**FX["default_config"], **{k: v for k, v in case["config"].items()
                                                                         if k not in ("id2label", "label2id")}})
        h = torch.tensor(case["hidden"])
        binary = "id2label" in case["config"]
        orig = (O.ci_encoder, O.na_encoder)
        O.ci_encoder = O.na_encoder = lambda p, cfg, batch, pre="": h
        try:
            p = {"logit_layer.weight": torch.tensor(case["weight"]), "logit_layer.bias": torch.tensor(case["bias"])}
            labels = torch.tensor(case["labels"], dtype=torch.float32 if binary else torch.long)
            em = torch.ones(h.shape[0], h.shape[1], dtype=torch.bool) if case["event_mask"] is None else \
                torch.tensor(case["event_mask"])
            pooling = cfg.task_specific_params["pooling_method"]
            loss, logits = O.stream_classification_loss(p, cfg, {"event_mask": em}, labels, pooling, binary)
        finally:
            O.ci_encoder, O.na_encoder = orig
        assert loss.item() == pytest.approx(case["want_loss"], rel=1e-6), case["msg"]
        assert torch.allclose(logits, torch.tensor(case["want_preds"])), case["msg"]


@pytest.mark.gpu
@pytest.mark.parametrize("pooling", ["cls", "last", "max", "mean"])
@pytest.mark.parametrize("binary", [False, True])
def test_fine_tuning_model_matches_oracle_f32(pooling, binary):
    """The real fine-tuning model on cuda (HIP encoder, f32) vs the oracle's restatement: loss and gradients."""
    import esgpt_oracle as O
    from eventstreamgpt_amd.synthetic import CONFIGS

    bc = CONFIGS["C1"]
    kw = dict(finetuning_task="t", task_specific_params={"pooling_method": pooling})
    if binary:
        kw.update(num_labels=2, id2label={0: "False", 1: "True"}, label2id={"False": 0, "True": 1})
    else:
        kw.update(num_labels=3)
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0, **kw)
    torch.manual_seed(0)
    m = ESTForStreamClassification(cfg).to("cuda")
    batch = bc.batch(0, batch_size=4)
    labels = torch.tensor([0.0, 1.0, 1.0, 0.0]) if binary else torch.tensor([0, 2, 1, 2])
    batch.stream_labels = {"t": labels}
    out = m(batch.to("cuda"))
    out.loss.backward()
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    p.update({k: v.detach().cpu() for k, v in m.named_buffers()})
    loss, logits = O.stream_classification_loss(p, cfg, batch, labels, pooling, binary)
    loss.backward()
    assert abs(out.loss.item() - loss.item()) <= 1e-5 * max(1.0, abs(loss.item()))
    assert torch.allclose(out.preds.detach().cpu(), logits.detach(), rtol=1e-4, atol=1e-5)
    for k, prm in m.named_parameters():
        if p[k].grad is None or prm.grad is None:
            continue
        ref = p[k].grad
        assert ((prm.grad.cpu() - ref).abs().max() / ref.abs().max().clamp_min(1e-12)).item() < 1e-4, k
