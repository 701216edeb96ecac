"""Data-dependent error semantics of the HIP path against the reference's exceptions, and the training step's
staging rules (HIP graphs per batch shape, stream labels, per-parameter AdamW steps, returned losses).

Reference behaviours:
* ``DataEmbeddingLayer._embed``: ``torch._assert(indices.max() < n_total_embeddings,
  f"Invalid embedding! {indices.max()} >= {n_total_embeddings}")`` (data_embedding_layer.py:485-488) — an
  AssertionError (``f"{indices.max()}"`` of a 0-dim tensor prints its value);
* ``get_TTE_outputs``: ``ValueError(f"NaNs in TTE_LL: {batch}")`` and ``ValueError(f"No observed time-to-event for
  >= 1 patient in batch: {batch}")`` (model_output.py:1360-1367), checked in that order;
* the reference raises before ``optimizer.step``: the parameters keep their values.
"""
import pytest
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.config import OptimizationConfig

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ci_model(name="C1", **kw):
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    cfg = CONFIGS[name].model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0, **kw)
    torch.manual_seed(0)
    return CIPPTForGenerativeSequenceModeling(cfg).to(DEV).train(), cfg


def _opt():
    return OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100)


@pytest.fixture(autouse=True)
def _clear():
    from eventstreamgpt_amd.kernels import err_word

    err_word(torch.device(DEV)).zero_()
    yield
    err_word(torch.device(DEV)).zero_()


@pytest.mark.parametrize("where", ["dynamic", "static"])
def test_bad_embedding_index_raises_reference_assert(where):
    from eventstreamgpt_amd.kernels import check_errors

    m, cfg = _ci_model()
    b = CONFIGS["C1"].batch(0, batch_size=4)
    V = cfg.vocab_size
    if where == "dynamic":
        b.dynamic_indices[1, 3, 0] = V + 7
        b.dynamic_indices[2, 5, 1] = V + 2
        want_max = b.dynamic_indices.max()
    else:
        b.static_indices[0, 1] = V + 3
        want_max = b.static_indices.max()
    m(b.to(DEV))
    with pytest.raises(AssertionError) as e:
        check_errors()
    assert str(e.value) == f"Invalid embedding! {want_max} >= {V}"
    check_errors()  # cleared: a second check passes


def test_tte_nan_raises_value_error():
    from eventstreamgpt_amd.kernels import check_errors

    m, _ = _ci_model()
    b = CONFIGS["C1"].batch(0, batch_size=4)
    b.time_delta[1, 2] = float("nan")
    bd = b.to(DEV)
    m(bd)
    with pytest.raises(ValueError) as e:
        check_errors(batch=bd)
    assert str(e.value) == f"NaNs in TTE_LL: {bd}"


def test_no_observed_tte_raises_value_error():
    from eventstreamgpt_amd.kernels import check_errors

    m, _ = _ci_model()
    b = CONFIGS["C1"].batch(0, batch_size=4)
    b.event_mask[2, 1:] = False  # one event: no observed time-to-event for subject 2
    bd = b.to(DEV)
    m(bd)
    with pytest.raises(ValueError) as e:
        check_errors(batch=bd)
    assert str(e.value) == f"No observed time-to-event for >= 1 patient in batch: {bd}"


@pytest.mark.parametrize("graph", [False, True])
def test_trainstep_error_skips_update_and_raises(graph):
    """A bad batch: AdamW leaves every parameter untouched (device-side guard) and the step raises the reference's
    exception no later than two steps on, or at ``check()``."""
    m, cfg = _ci_model()
    bc = CONFIGS["C1"]
    ts = TrainStep(m, _opt(), torch.bfloat16, use_graph=graph)
    ts.step(bc.batch(0, batch_size=8, device=DEV).packed())
    ts.check()
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    bad = bc.batch(1, batch_size=8)
    bad.dynamic_indices[0, 0, 0] = cfg.vocab_size
    # f"{indices.max()}" of a 0-dim tensor formats its value: "Invalid embedding! 69 >= 69"
    with pytest.raises(AssertionError, match=f"^Invalid embedding! {cfg.vocab_size} >= {cfg.vocab_size}$"):
        ts.step(bad.to(DEV).packed())
        ts.check()
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    # training continues normally after the error was raised
    ts.step(bc.batch(2, batch_size=8, device=DEV).packed())
    ts.check()
    assert any(not torch.equal(v, before[k]) for k, v in m.state_dict().items())


def test_trainstep_raises_without_explicit_check():
    m, cfg = _ci_model()
    bc = CONFIGS["C1"]
    ts = TrainStep(m, _opt(), torch.bfloat16, use_graph=True)
    bad = bc.batch(1, batch_size=8)
    bad.dynamic_indices[3, 2, 1] = cfg.vocab_size + 1
    good = [bc.batch(i, batch_size=8, device=DEV).packed() for i in (2, 3, 4)]
    with pytest.raises(AssertionError, match="Invalid embedding!"):
        ts.step(good[0])
        ts.step(bad.to(DEV).packed())
        for g in good:  # raised when the step after next is submitted
            ts.step(g)


@pytest.mark.parametrize("graph", [False, True])
def test_trainstep_error_discards_queued_steps(graph):
    """A good step queued behind a bad one (submitted before the bad step's flags were read) is discarded too: after
    the raise the parameters are the pre-error values, the AdamW / LR counters are those of the last good step, and
    training resumes exactly like a run that never saw the bad batch and its follower."""
    bc = CONFIGS["C1"]
    good = [bc.batch(i, batch_size=8, device=DEV).packed() for i in (0, 2, 3)]

    def fresh():
        m, cfg = _ci_model()
        return m, cfg, TrainStep(m, _opt(), torch.bfloat16, use_graph=graph)

    m, cfg, ts = fresh()
    bad = bc.batch(1, batch_size=8)
    bad.dynamic_indices[1, 1, 0] = cfg.vocab_size + 3
    ts.step(good[0])
    ts.check()
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    steps_before, sched_before = list(ts.opt.steps), ts.sched_step
    with pytest.raises(AssertionError, match="Invalid embedding!"):
        ts.step(bad.to(DEV).packed())
        ts.step(good[1])  # queued behind the bad step: discarded with it
        ts.check()
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert ts.opt.steps == steps_before and ts.sched_step == sched_before
    ts.step(good[2])
    ts.check()
    after = {k: v.detach().clone() for k, v in m.state_dict().items()}

    m2, _, ts2 = fresh()  # the same run without the bad batch and its follower
    ts2.step(good[0])
    ts2.step(good[2])
    ts2.check()
    for k, v in m2.state_dict().items():
        assert torch.equal(v, after[k]), k


def test_graph_per_shape_signature_matches_eager():
    """Batches of different shapes (B, L, M, S including a size-1 S) under use_graph: one graph per signature, no
    broadcasting into a captured buffer; losses and parameters equal the eager run's."""
    bc = CONFIGS["C1"]
    shapes = []
    for i, (B, S) in enumerate([(8, 2), (6, 2), (8, 1), (8, 2), (6, 2), (8, 1)]):
        b = bc.batch(i, batch_size=B)
        b.static_indices = b.static_indices[:, :S].contiguous()
        b.static_measurement_indices = b.static_measurement_indices[:, :S].contiguous()
        shapes.append(b.to(DEV).packed())

    def run(graph):
        m, _ = _ci_model()
        ts = TrainStep(m, _opt(), torch.bfloat16, use_graph=graph)
        losses = [ts.step(b) for b in shapes]
        ts.check()
        return [float(x) for x in losses], {k: v.detach().clone() for k, v in m.state_dict().items()}, ts

    le, se, _ = run(False)
    lg, sg, ts = run(True)
    assert len(ts.graphs) == 3
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg)
    for k in se:
        assert (sg[k].float() - se[k].float()).abs().max().item() < 1e-4, k


def test_graph_losses_are_not_aliased():
    """step() returns a fresh tensor per step in graph mode too (the static loss is overwritten by each replay)."""
    m, _ = _ci_model()
    bc = CONFIGS["C1"]
    ts = TrainStep(m, _opt(), torch.bfloat16, use_graph=True)
    losses = [ts.step(bc.batch(i, batch_size=8, device=DEV).packed()) for i in range(3)]
    ts.check()
    vals = [float(x) for x in losses]
    assert len(set(vals)) == 3


@pytest.mark.parametrize("graph", [False, True])
def test_fine_tuning_head_trainstep_graph_matches_eager(graph):
    """ESTForStreamClassification under TrainStep: the stream labels of every batch are staged into the graph (a
    graph replaying the first batch's labels would give different losses)."""
    from eventstreamgpt_amd.transformer.fine_tuning_model import ESTForStreamClassification

    bc = CONFIGS["C1"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0, finetuning_task="t",
                          task_specific_params={"pooling_method": "mean"}, num_labels=3)
    batches = []
    for i in range(4):
        b = bc.batch(i, batch_size=8)
        b.stream_labels = {"t": torch.randint(0, 3, (8,), generator=torch.Generator().manual_seed(i))}
        batches.append(b.to(DEV).packed())

    def run(use_graph):
        torch.manual_seed(0)
        m = ESTForStreamClassification(cfg).to(DEV).train()
        ts = TrainStep(m, _opt(), torch.bfloat16, use_graph=use_graph)
        out = [float(ts.step(b)) for b in batches]
        ts.check()
        return out, ts.use_graph

    le, _ = run(False)
    lg, used = run(graph)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg, used)


def test_fused_adamw_per_parameter_steps():
    """torch.optim.AdamW keeps one step count per parameter: a parameter that skips a step gets its own bias
    correction afterwards (esgpt_adamw's per-tensor table)."""
    from eventstreamgpt_amd.train import FusedAdamW

    g = torch.Generator().manual_seed(0)
    shapes = [(300, 64), (7,), (4099,)]
    base = [torch.randn(s, generator=g) for s in shapes]
    pa = [b.clone().to(DEV).requires_grad_(True) for b in base]
    pb = [b.clone().to(DEV).requires_grad_(True) for b in base]
    oa = FusedAdamW(pa, lr=1e-2, weight_decay=0.01)
    ob = torch.optim.AdamW(pb, lr=1e-2, weight_decay=0.01)
    skip = {1: {0, 1}, 2: {2}}  # param -> steps without gradient
    for step in range(5):
        for i, (a, b) in enumerate(zip(pa, pb)):
            if step in skip.get(i, ()):
                a.grad = b.grad = None
                continue
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad, b.grad = gr.clone(), gr.clone()
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        assert (a.detach() - b.detach()).abs().max().item() <= 1e-6 * max(1.0, b.abs().max().item())
    assert oa.steps == [int(ob.state[p]["step"]) for p in pb]
