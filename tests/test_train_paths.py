"""Training-step host logic and paths beyond the fused CI graph: the LR schedule against transformers' own, the
strict batch staging a captured graph relies on, reference error semantics of the input layer, and the
nested-attention step (bf16 HIP blocks) against the module path and the reference's loss."""
import pytest
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep, graph_safe
from eventstreamgpt_amd.transformer.config import OptimizationConfig


def test_graph_safe_selection():
    ci = CONFIGS["C1"].model_config()
    na = CONFIGS["C4"].model_config()
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    assert graph_safe(CIPPTForGenerativeSequenceModeling(ci))
    assert graph_safe(CIPPTForGenerativeSequenceModeling(ci), torch.float32)
    assert graph_safe(NAPPTForGenerativeSequenceModeling(na))  # bf16: fused NA blocks
    assert not graph_safe(NAPPTForGenerativeSequenceModeling(na), torch.float32)  # module path stays eager


@pytest.mark.parametrize("warm,total,power,init,end", [(10, 100, 1.0, 1e-3, 0.0), (0, 50, 2.0, 1e-2, 1e-5),
                                                      (7, 8, 1.0, 1e-3, 1e-7), (3, 40, 0.5, 5e-4, 1e-6)])
def test_poly_decay_matches_transformers(warm, total, power, init, end):
    """poly_decay_lambda vs transformers.get_polynomial_decay_schedule_with_warmup (configure_optimizers,
    generative_modeling.py:467-473) over warm-up, decay and the tail past max_training_steps."""
    from transformers import get_polynomial_decay_schedule_with_warmup

    from eventstreamgpt_amd.train import poly_decay_lambda

    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=init)
    sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=warm, num_training_steps=total,
                                                      power=power, lr_end=end)
    f = poly_decay_lambda(warm, total, power, init, end)
    for step in range(total + 6):
        assert init * f(step) == pytest.approx(opt.param_groups[0]["lr"], rel=1e-12, abs=1e-18), step
        opt.step()
        sched.step()


def test_poly_decay_rejects_end_above_init():
    from transformers import get_polynomial_decay_schedule_with_warmup

    from eventstreamgpt_amd.train import poly_decay_lambda

    opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=1e-3)
    with pytest.raises(ValueError) as want:
        get_polynomial_decay_schedule_with_warmup(opt, 1, 10, lr_end=1e-2)
    with pytest.raises(ValueError) as got:
        poly_decay_lambda(1, 10, 1.0, 1e-3, 1e-2)
    assert str(got.value) == str(want.value)


def test_batch_copy_requires_same_shapes():
    """Staging into a captured graph's static batch: a batch of another shape signature raises instead of
    broadcasting (a size-1 static dimension would otherwise duplicate entries into every slot)."""
    bc = CONFIGS["C1"]
    a = bc.batch(0, batch_size=4).packed()
    b = bc.batch(1, batch_size=4).packed()
    assert a.shape_signature() == b.shape_signature()
    a.copy_(b)
    assert torch.equal(a.dynamic_indices, b.dynamic_indices) and torch.equal(a.static_indices, b.static_indices)
    c = bc.batch(1, batch_size=4)
    c.static_indices = c.static_indices[:, :1].contiguous()
    c.static_measurement_indices = c.static_measurement_indices[:, :1].contiguous()
    with pytest.raises(ValueError, match="shape signature"):
        a.copy_(c)
    d = bc.batch(2, batch_size=3)
    with pytest.raises(ValueError, match="shape signature"):
        a.copy_(d)


def test_batch_packed_copies_stream_labels():
    """packed() owns its stream labels and copy_ stages them (the fine-tuning head reads them inside a graph)."""
    bc = CONFIGS["C1"]
    a = bc.batch(0, batch_size=4)
    a.stream_labels = {"t": torch.tensor([0, 1, 2, 1])}
    s = a.packed()
    assert s.stream_labels["t"].data_ptr() != a.stream_labels["t"].data_ptr()
    b = bc.batch(1, batch_size=4).packed()
    b.stream_labels = {"t": torch.tensor([2, 2, 0, 0])}
    s.copy_(b)
    assert torch.equal(s.stream_labels["t"], b.stream_labels["t"])


def test_empty_measurement_group_raises_in_forward():
    """The reference raises the empty-group ValueError in forward (data_embedding_layer.py:529-535), not at
    construction; same type and message here."""
    from eventstreamgpt_amd.data.data_embedding_layer import DataEmbeddingLayer

    layer = DataEmbeddingLayer(10, 8, "drop", categorical_embedding_dim=4, numerical_embedding_dim=4,
                               split_by_measurement_indices=[[], [1], []])
    want = ("Empty measurement index group: [] at index 2! Only the first (i=0) group can be empty (in cases where "
            "there are no FUNCTIONAL_TIME_DEPENDENT measurements).")
    with pytest.raises(ValueError) as e:
        layer(CONFIGS["C1"].batch(0, batch_size=2))
    assert str(e.value) == want


@pytest.mark.gpu
def test_nested_attention_eager_steps_deterministic():
    """The NA training step (eager) is run-to-run deterministic and finite over several optimizer steps."""
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS["C4"]
    batches = [bc.batch(i, batch_size=2, device="cuda").packed() for i in range(4)]
    losses = {}
    for run in (0, 1):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                       torch.bfloat16, use_graph=False)
        losses[run] = [float(ts.step(b)) for b in batches]
        ts.check()
        assert all(torch.isfinite(p).all() for p in m.parameters())
    assert all(abs(a - b) < 1e-4 * max(1.0, abs(a)) for a, b in zip(losses[0], losses[1]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["na_small", "na_joint_attn"])
def test_nested_attention_bf16_fused_blocks_match_module_path(name):
    """bf16: the NA blocks through the HIP kernels (fused.inner_block_fused) against the PyTorch module path, and the
    loss against the reference's f32 golden value (bf16 tolerance)."""
    from helpers import load_case

    from eventstreamgpt_amd import fused
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    fx, cfg, batch = load_case(name)
    b = batch.to("cuda")
    res = {}
    for enabled in (True, False):
        fused.ENABLED = enabled
        try:
            m = NAPPTForGenerativeSequenceModeling(cfg)
            m.load_state_dict(fx["state_dict"])
            m = m.cuda().train()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(b)
            out.loss.backward()
            res[enabled] = (float(out.loss), {k: p.grad.detach().float().clone() for k, p in m.named_parameters()
                                              if p.grad is not None})
        finally:
            fused.ENABLED = True
    (lf, gf), (lm, gm) = res[True], res[False]
    want = float(fx["loss"])
    assert abs(lf - want) <= 2e-2 * abs(want), (lf, want)
    assert abs(lf - lm) <= 2e-2 * abs(lm), (lf, lm)
    assert set(gf) == set(gm)
    for k in gm:
        scale = gm[k].abs().max().clamp_min(1e-6)
        assert torch.isfinite(gf[k]).all(), k
        assert ((gf[k] - gm[k]).abs().max() / scale).item() < 0.1, k


@pytest.mark.gpu
def test_nested_attention_graph_replay_matches_eager_with_allocations_between_replays():
    """The NA training step captured as a HIP graph (graph_safe: NA in bf16 is captured by default) replays with
    fresh batches while the host allocates and frees device memory between replays (so a buffer the graph uses but
    does not own would be reused and corrupted), and matches eager steps: losses every step, parameters after."""
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS["C4"]
    batches = [bc.batch(i, batch_size=4, device="cuda").packed() for i in range(5)]

    def run(graph):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=2, max_training_steps=100),
                       torch.bfloat16, use_graph=graph)
        losses, junk = [], []
        for i, b in enumerate(batches):
            losses.append(float(ts.step(b)))
            # host-side allocations between replays: reuse any freed block a captured kernel still points at
            junk = [torch.full((1 << (16 + (i + j) % 6),), float(j + 1), device="cuda") for j in range(24)]
            torch.cuda.synchronize()
            del junk
        ts.check()
        return losses, {k: v.detach().float().clone() for k, v in m.state_dict().items()}, ts.use_graph

    le, se, _ = run(False)
    lg, sg, used = run(True)
    assert used
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg)
    for k in se:
        assert (sg[k] - se[k]).abs().max().item() < 1e-4, k


@pytest.mark.gpu
def test_replayed_losses_held_across_steps():
    """The replayed step hands back its loss through the optimizer launch's hand-off ring (with the optimizer
    launched after the replay, and captured at the end of the step's graph, TrainStep.fuse_optimizer): losses held
    unread across later replays — more of them than the ring has entries — keep their own step's value, equal bitwise
    to the pack-launch copy's and to what each step returned when read at once; the parameters after the steps are
    bitwise equal too."""
    from eventstreamgpt_amd import train as train_mod
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C2"]
    batches = [bc.batch(i, batch_size=8, device="cuda").packed() for i in range(6)]

    def run(fuse, read_now, ring_len=4, alias=None):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=2, max_training_steps=100),
                       torch.bfloat16, use_graph=True, fuse_optimizer=fuse is True)
        ts.ring_len = ring_len
        saved = train_mod.LOSS_IN_OPT
        train_mod.LOSS_IN_OPT = bool(fuse)  # "ring": host-launched optimizer, loss through its ring entry
        try:
            if alias is not None:  # aliases of the returned loss (not the object itself) held across the ring
                held = [alias(ts.step(b)) for b in batches]
            else:
                held = [ts.step(b) for b in batches] if not read_now else [float(ts.step(b)) for b in batches]
        finally:
            train_mod.LOSS_IN_OPT = saved
        ts.check()
        assert ts.use_graph
        assert all(e[4] == ("fused" if fuse is True else None) for e in ts.graphs.values() if e is not None)
        return [x if isinstance(x, float) else float(x.reshape(())) for x in held], [p.detach().clone() for p in m.parameters()]

    a, pa = run(True, False)
    for fuse in (True, "ring"):
        for alias in (lambda x: x.detach(), lambda x: x.view(1), lambda x: x[None]):
            assert run(fuse, False, alias=alias)[0] == a
    b, pb = run(False, False)
    c, _ = run(True, True, ring_len=64)
    d, pd = run("ring", False)
    assert a == b == c == d
    assert all(torch.equal(x, y) for x, y in zip(pa, pd))
    assert len(set(a)) == len(a), a  # every step's own value, not a later replay's
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))


def _na_graph_vs_eager(batches, fused_enabled=True):
    from eventstreamgpt_amd import fused
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS["C4"]

    def run(graph):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                       torch.bfloat16, use_graph=graph, _force_graph=graph and not fused_enabled)
        losses = [float(ts.step(b)) for b in batches]
        ts.check()
        return losses, {k: v.detach().float().clone() for k, v in m.state_dict().items()}, ts

    old = fused.ENABLED
    fused.ENABLED = fused_enabled
    try:
        le, se, _ = run(False)
        lg, sg, ts = run(True)
    finally:
        fused.ENABLED = old
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg)
    for k in se:
        assert (sg[k] - se[k]).abs().max().item() < 1e-4, k
    return ts


@pytest.mark.gpu
def test_ragged_token_counts_stay_on_library_gemms_and_capture():
    """A batch with a token count that is not a multiple of 8 (B·L = 253; the reference pads each batch to its own
    longest subject, pytorch_dataset.py:571) runs the fused NA blocks on the library GEMMs (the dW products take any
    token count; edge rows are zero-filled in-kernel): its warm-up shows no ATen GEMM or reduction, so the signature is
    captured, and graph replay equals the eager step."""
    bc = CONFIGS["C4"]
    odd = [bc.batch(i, batch_size=1, device="cuda")[:, :253].packed() for i in range(3)]  # 253 tokens
    even = [bc.batch(10 + i, batch_size=2, device="cuda").packed() for i in range(2)]
    ts = _na_graph_vs_eager(odd + even)
    assert ts.graphs[odd[0].shape_signature()] is not None, ts.capture_report
    assert not ts.capture_report[odd[0].shape_signature()], ts.capture_report
    assert ts.graphs[even[0].shape_signature()] is not None, ts.capture_report


@pytest.mark.gpu
def test_graph_capture_skips_signatures_with_aten_gemm_fallback():
    """The module-by-module path (fused.ENABLED off) runs its Linears through PyTorch-ROCm BLAS, whose backward
    replayed from a HIP graph returns wrong bias gradients (tools/graph_blaslt_repro.py): TrainStep does not capture
    such a signature (warm-up under _GemmSpy) and runs it eagerly, with eager's losses and parameters."""
    bc = CONFIGS["C4"]
    batches = [bc.batch(i, batch_size=1, device="cuda").packed() for i in range(3)]
    ts = _na_graph_vs_eager(batches, fused_enabled=False)
    sig = batches[0].shape_signature()
    assert ts.graphs[sig] is None and ts.capture_report[sig]


@pytest.mark.gpu
def test_step_error_flags_are_per_step():
    """A step whose batch holds an out-of-range embedding index is a no-op for the parameters (its AdamW sees the
    flag). On the device each step's first launch starts its own flags and moves the previous step's into the sticky
    word, so every later step stays a no-op until the host has read and cleared the block (device semantics,
    TrainStep(check_errors=False): kernels.check_errors raises the reference's AssertionError and clears it; then
    steps update again, with clear flags of their own). With checking on, the error is raised at a later submission
    and the failing step's AdamW / LR-schedule counters are rolled back."""
    from eventstreamgpt_amd.kernels import check_errors, err_word
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C1"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    good = [bc.batch(i, batch_size=4, device="cuda").packed() for i in range(3)]
    bad = bc.batch(7, batch_size=4, device="cuda").packed()
    bad.dynamic_indices[0, 0, 0] = cfg.vocab_size + 5
    opt_cfg = OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=0, max_training_steps=100)

    def snap(m):
        return {k: v.detach().clone() for k, v in m.named_parameters()}

    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
    ts = TrainStep(m, opt_cfg, torch.bfloat16, use_graph=False, check_errors=False)
    ts.step(good[0])
    p0 = snap(m)
    ts.step(bad)
    p1 = snap(m)
    assert all(torch.equal(p0[k], p1[k]) for k in p0)  # the failing step did not update
    ts.step(good[1])
    p2 = snap(m)
    assert all(torch.equal(p1[k], p2[k]) for k in p0)  # nor did the step queued behind it (sticky word)
    w = err_word(torch.device("cuda"))
    assert int(w[0]) & 0xFFFFFFFF == 0 and int(w[0]) >> 32 != 0  # its own flags are clear, the sticky word set
    with pytest.raises(AssertionError, match="Invalid embedding!"):
        check_errors(torch.device("cuda"), cfg.vocab_size)  # reads and clears the block
    ts.step(good[2])
    p3 = snap(m)
    assert any(not torch.equal(p2[k], p3[k]) for k in p0)  # the next step updates
    assert int(err_word(torch.device("cuda"))[0]) == 0

    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
    ts = TrainStep(m, opt_cfg, torch.bfloat16, use_graph=False)
    ts.step(good[0])
    ts.step(bad)
    torch.cuda.synchronize()
    assert ts.sched_step == 2 and {s for s in ts.opt.steps if s} == {2}
    with pytest.raises(AssertionError, match="Invalid embedding!"):
        ts.step(good[1])
    assert ts.sched_step == 1 and {s for s in ts.opt.steps if s} == {1}
    ts.step(good[2])  # training continues from the rolled-back counters
    ts.check()
    assert ts.sched_step == 2 and {s for s in ts.opt.steps if s} == {2}


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [True, False])
def test_weight_grad_overlap_matches_serial_step(graph):
    """TrainStep with the projections' weight gradients on the second stream (overlap_weight_grads) vs one stream: the same
    losses and parameters bit for bit over several steps, captured as a HIP graph or eager (the CI model at the
    C2 widths, reduced batch)."""
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C2"]
    batches = [bc.batch(i, batch_size=4, device="cuda").packed() for i in range(4)]

    def run(overlap):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                       torch.bfloat16, use_graph=graph, overlap_weight_grads=overlap)
        losses = [float(ts.step(b)) for b in batches]
        ts.check()
        return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}

    l0, s0 = run(False)
    l1, s1 = run(True)
    assert l0 == l1
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("cfg_name", ["C2", "C4"])
def test_deferred_colsums_match_per_layer_sums(graph, cfg_name):
    """TrainStep with the LayerNorm column sums deferred to one esgpt::colsum_flush per backward (the default) vs
    one sum launch per LayerNorm: the same losses and parameters bit for bit (CI at the C2 widths, NA at C4; HIP
    graph and eager)."""
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS[cfg_name]
    Model = CIPPTForGenerativeSequenceModeling if cfg_name == "C2" else NAPPTForGenerativeSequenceModeling
    batches = [bc.batch(i, batch_size=2, device="cuda").packed() for i in range(3)]

    def run(defer):
        cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
        torch.manual_seed(0)
        m = Model(cfg).cuda().train()
        from eventstreamgpt_amd.kernels import _seed_counter

        _seed_counter(torch.device("cuda")).zero_()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                       torch.bfloat16, use_graph=graph, defer_colsums=defer)
        losses = [float(ts.step(b)) for b in batches]
        ts.check()
        return losses, {k: v.detach().clone() for k, v in m.state_dict().items()}

    l0, s0 = run(False)
    l1, s1 = run(True)
    assert l0 == l1
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_bench_configs_capture_without_aten_gemm_or_reduction(name):
    """The bench configurations' steps are captured (one HIP graph per signature) and their warm-up pass runs no ATen
    GEMM and no ATen reduction (a captured reduction's semaphore memset does not replay correctly: DESIGN.md §5)."""
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS[name]
    cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
    Model = (CIPPTForGenerativeSequenceModeling if cfg.structured_event_processing_mode == "conditionally_independent"
             else NAPPTForGenerativeSequenceModeling)
    torch.manual_seed(0)
    m = Model(cfg).cuda().train()
    ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                   torch.bfloat16, use_graph=True)
    b = bc.batch(0, batch_size=2, device="cuda").packed()
    assert torch.isfinite(ts.step(b)).all()
    ts.check()
    sig = b.shape_signature()
    assert ts.capture_report[sig] == [], ts.capture_report
    assert ts.graphs[sig] is not None


@pytest.mark.gpu
def test_nested_attention_input_dropout_kernel():
    """The NA input layer's embedding_dropout (nn.Dropout, transformer.py:900-936) runs as the library's
    counter-hash dropout (esgpt::residual without x): out = embed · keep / (1 - p), keep ≈ 1 - p of the elements, the
    same keep mask in the backward; identity in eval mode."""
    from eventstreamgpt_amd.transformer.transformer import NestedAttentionPointProcessInputLayer

    bc = CONFIGS["C4"]
    p = 0.3
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=p, resid_dropout=0.0)
    torch.manual_seed(0)
    layer = NestedAttentionPointProcessInputLayer(cfg).cuda().train()
    b = bc.batch(0, batch_size=4, device="cuda")
    out = layer(b)
    emb = layer.data_embedding_layer.embed(b, time_layer=layer.time_embedding_layer, cumsum=True).detach()
    assert out.shape == emb.shape
    live = emb != 0
    keep = (out != 0) & live
    frac = keep.sum().item() / live.sum().item()
    assert abs(frac - (1 - p)) < 0.01, frac
    torch.testing.assert_close(out.detach()[keep], emb[keep] / (1 - p), rtol=1e-6, atol=0)
    assert (out.detach()[live & ~keep] == 0).all()
    # backward: the same keep mask and scale (the op's own gradient w.r.t. its input)
    from eventstreamgpt_amd import fused

    x = emb.clone().requires_grad_(True)
    torch.manual_seed(1)
    y = fused.residual(None, x, None, 1, 0, p).view(x.shape)
    g = torch.randn_like(y)
    y.backward(g)
    kept = (y.detach() != 0) & (x.detach() != 0)
    torch.testing.assert_close(x.grad[kept], g[kept] / (1 - p), rtol=1e-6, atol=0)
    assert (x.grad[(x.detach() != 0) & ~kept] == 0).all()
    layer.eval()
    torch.testing.assert_close(layer(b), emb, rtol=0, atol=0)


@pytest.mark.gpu
def test_device_lr_schedule_matches_host_schedule():
    """The optimizer step's lr and bias corrections computed on the device (esgpt_adamw_prepare) equal the host
    restatement of transformers' polynomial decay with warmup (LambdaLR step counting) and torch's per-parameter
    bias corrections, over warmup, decay and past-the-end steps; a parameter without a gradient keeps its count."""
    from eventstreamgpt_amd.train import FusedAdamW, poly_decay_lambda

    warm, total, power, init, end = 3, 10, 2.0, 1e-3, 1e-5
    lam = poly_decay_lambda(warm, total, power, init, end)
    p = [torch.zeros(8, device="cuda", requires_grad=True), torch.zeros(3, device="cuda", requires_grad=True)]
    opt = FusedAdamW(p, lr=init)
    opt.schedule = (1, warm, total, power, init, end)
    steps = [0, 0]
    for k in range(14):
        p[0].grad = torch.ones_like(p[0])
        p[1].grad = torch.ones_like(p[1]) if k % 3 else None  # skipped on some steps
        opt.step()
        for i in range(2):
            if p[i].grad is not None:
                steps[i] += 1
        lr = init * lam(k)
        assert abs(float(opt._lr_dev) - lr) <= 1.2e-7 * lr + 1e-30, (k, float(opt._lr_dev), lr)  # f32 rounding
        per = opt._plan()["per"].cpu().tolist()
        for t, i in enumerate(opt._active):
            want = [lr / (1.0 - 0.9 ** steps[i]), (1.0 - 0.999 ** steps[i]) ** 0.5]
            assert abs(per[2 * t] - want[0]) <= 1e-6 * want[0] and abs(per[2 * t + 1] - want[1]) <= 1e-6 * want[1]
    assert opt._counters.tolist() == steps + [14] and opt.steps == steps


@pytest.mark.gpu
def test_captured_optimizer_step_matches_host_launched():
    """The optimizer step captured at the end of the step's graph (the default, fuse_optimizer) and replayed as its
    own graph (capture_optimizer=True) — lr / bias corrections from the device counters in both — give bit-identical
    parameters and step counts to the host-launched device step."""
    bc = CONFIGS["C1"]
    batches = [bc.batch(i, batch_size=8, device="cuda").packed() for i in range(4)]
    out = {}
    for mode in ("host", "own-graph", "fused"):
        from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=2, max_training_steps=10),
                       torch.bfloat16, use_graph=True, capture_optimizer=mode == "own-graph",
                       fuse_optimizer=mode == "fused")
        for b in batches:
            ts.step(b)
        ts.check()
        kinds = {type(e[4]).__name__ if not isinstance(e[4], str) else e[4] for e in ts.graphs.values() if e is not None}
        assert kinds == {"host": {"NoneType"}, "own-graph": {"CUDAGraph"}, "fused": {"fused"}}[mode], kinds
        out[mode] = ({k: v.detach().clone() for k, v in m.state_dict().items()}, list(ts.opt.steps),
                     ts.opt._counters.tolist())
    for mode in ("own-graph", "fused"):
        for k in out["host"][0]:
            assert torch.equal(out["host"][0][k], out[mode][0][k]), (mode, k)
        assert out["host"][1] == out[mode][1] and out["host"][2] == out[mode][2]


def test_hand_off_ring_claims_cpu():
    """The optimizer hand-off ring's host side (TrainStep._claim / _unclaim / _ring_loss): an entry whose storage the
    caller still shares when it comes round again — through the returned object or any alias of it (detach, view,
    index) — gets a fresh allocation and its table slot is re-pointed, so the held values never change; an entry
    nobody holds is reused as is; a claim with no launch behind it is taken back."""
    m = torch.nn.Linear(3, 2)
    ts = TrainStep(m, OptimizationConfig(init_lr=1e-3), compute_dtype=torch.float32)
    ts.ring_len = 3
    like = torch.zeros(())
    _, _, tab, _ = ts._ring_state()
    kept = []
    for alias in (lambda x: x, lambda x: x.detach(), lambda x: x.view(1)[None]):
        s = ts._claim()
        ts._slots[s][0] = 10.0 + s  # what the launch would write
        kept.append(alias(ts._ring_loss(s, like)))
    assert [ts._slots[i].data_ptr() for i in range(3)] == tab.tolist()
    for i in range(3):  # every entry comes round again while an alias of its loss is held: fresh allocations
        s = ts._claim()
        assert s == i and ts._slots[s].data_ptr() == int(tab[s]) and ts._slots[s].data_ptr() != kept[i].data_ptr()
        ts._slots[s][0] = -1.0
    assert [float(k.reshape(())) for k in kept] == [10.0, 11.0, 12.0]
    kept.clear()  # nothing held any more: the entries are reused in place
    before = tab.tolist()
    for i in range(3):
        ts._ring_loss(ts._claim(), like)
    assert tab.tolist() == before
    s = ts._claim()
    ts._unclaim()  # (no launch followed)
    assert ts._claim() == s


def test_gradient_accumulation_single_process_cpu():
    """OptimizationConfig.gradient_accumulation = 3 (Lightning's accumulate_grad_batches, generative_modeling.py:661-664)
    without DDP: the optimizer and the LR schedule step once per 3 batches on the sum of the 3 batches' gradients of
    loss / 3; a parameter that receives no gradient in a window is skipped."""
    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(6, 5)
            self.b = torch.nn.Linear(5, 3)
            self.unused = torch.nn.Linear(2, 2)

        def forward(self, x):
            class Out:
                pass

            o = Out()
            o.loss = self.b(torch.tanh(self.a(x))).pow(2).mean()
            return o

    from eventstreamgpt_amd.train import poly_decay_lambda

    def data(i):
        return torch.randn(4 + i, 6, generator=torch.Generator().manual_seed(77 + i))

    k, windows = 3, 2
    cfg = OptimizationConfig(init_lr=0.05, lr_num_warmup_steps=1, max_training_steps=8, gradient_accumulation=k)
    torch.manual_seed(0)
    m = Toy()
    ts = TrainStep(m, cfg, compute_dtype=torch.float32)
    losses = []
    for i in range(k * windows):
        losses.append(float(ts.step(data(i))))
        assert ts.sched_step == (i + 1) // k
    torch.manual_seed(0)
    ref = Toy()
    opt = torch.optim.AdamW(ref.parameters(), lr=cfg.init_lr, weight_decay=cfg.weight_decay)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, poly_decay_lambda(1, 8, 1.0, cfg.init_lr, cfg.end_lr))
    for w in range(windows):
        opt.zero_grad(set_to_none=True)
        for i in range(w * k, (w + 1) * k):
            loss = ref(data(i)).loss
            assert float(loss) == pytest.approx(losses[i], rel=1e-6)
            (loss / k).backward()
        opt.step()
        sched.step()
    for (name, a), b in zip(m.state_dict().items(), ref.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7, msg=name)
    assert m.unused.weight.grad is None  # never touched: AdamW skipped it, as torch does


def test_gradient_accumulation_partial_window_flush_cpu():
    """After the window's optimizer step the gradients it read stay readable (the buffer is zeroed at the start of
    the next window, not right after the step), and ``flush()`` applies an incomplete last window as Lightning does
    (each batch's loss scaled by 1 / k whatever the window's length)."""
    from eventstreamgpt_amd.train import poly_decay_lambda

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(6, 5)

        def forward(self, x):
            class Out:
                pass

            o = Out()
            o.loss = torch.tanh(self.a(x)).pow(2).mean()
            return o

    def data(i):
        return torch.randn(3 + i, 6, generator=torch.Generator().manual_seed(5 + i))

    k = 3
    cfg = OptimizationConfig(init_lr=0.05, lr_num_warmup_steps=1, max_training_steps=8, gradient_accumulation=k)
    torch.manual_seed(0)
    m = Toy()
    ts = TrainStep(m, cfg, compute_dtype=torch.float32)
    for i in range(k):
        ts.step(data(i))
    g_after = m.a.weight.grad.clone()
    assert g_after.abs().sum() > 0  # still the window's sums after the step that consumed them
    assert not ts.flush()  # nothing pending
    for i in range(k, k + 2):  # an incomplete window of 2
        ts.step(data(i))
    assert ts.sched_step == 1 and ts.flush() and ts.sched_step == 2
    torch.manual_seed(0)
    ref = Toy()
    opt = torch.optim.AdamW(ref.parameters(), lr=cfg.init_lr, weight_decay=cfg.weight_decay)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, poly_decay_lambda(1, 8, 1.0, cfg.init_lr, cfg.end_lr))
    for win in (range(0, k), range(k, k + 2)):
        opt.zero_grad(set_to_none=True)
        for i in win:
            (ref(data(i)).loss / k).backward()
        if win.start == 0:
            torch.testing.assert_close(ref.a.weight.grad, g_after, rtol=1e-6, atol=1e-7)
        opt.step()
        sched.step()
    for (name, a), b in zip(m.state_dict().items(), ref.state_dict().values()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7, msg=name)


def test_warmup_not_below_total_schedule():
    """lr_num_warmup_steps >= max_training_steps: the reference schedule never reaches its decay branch when warmup
    exceeds total, and divides 0 / 0 at step == warmup == total (transformers raises ZeroDivisionError there)."""
    from transformers import get_polynomial_decay_schedule_with_warmup

    from eventstreamgpt_amd.train import poly_decay_lambda

    f = poly_decay_lambda(6, 4, 1.0, 1e-3, 1e-6)
    opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=1e-3)
    sched = get_polynomial_decay_schedule_with_warmup(opt, num_warmup_steps=6, num_training_steps=4, lr_end=1e-6)
    for step in range(10):
        assert 1e-3 * f(step) == pytest.approx(opt.param_groups[0]["lr"], rel=1e-12), step
        opt.step()
        sched.step()
    g = poly_decay_lambda(3, 3, 1.0, 1e-3, 1e-6)
    with pytest.raises(ZeroDivisionError):
        g(3)


@pytest.mark.gpu
def test_gradient_accumulation_graph_matches_eager_and_reference():
    """gradient_accumulation = 2 on the GPU: the HIP-graph step (gradients summed into the window buffer after each
    replay) equals the eager step, and both equal a hand-written loop (backward of loss / 2 per batch, summed
    gradients, FusedAdamW at the schedule's lr once per window)."""
    from eventstreamgpt_amd.train import FusedAdamW
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C1"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    opt_cfg = OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=50, gradient_accumulation=2)
    batches = [bc.batch(s, batch_size=8, device="cuda:0").packed() for s in range(4)]

    def run(graph):
        torch.manual_seed(0)
        m = CIPPTForGenerativeSequenceModeling(cfg).to("cuda:0").train()
        ts = TrainStep(m, opt_cfg, torch.bfloat16, use_graph=graph)
        for b in batches:
            ts.step(b)
        ts.check()
        assert ts.sched_step == 2 and {s for s in ts.opt.steps if s} == {2}
        return {k: v.detach().clone() for k, v in m.state_dict().items()}

    got_graph, got_eager = run(True), run(False)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).to("cuda:0").train()
    params = [p for p in m.parameters() if p.requires_grad]
    opt = FusedAdamW(params, lr=opt_cfg.init_lr, weight_decay=opt_cfg.weight_decay)
    from eventstreamgpt_amd.train import poly_decay_lambda

    lam = poly_decay_lambda(1, 50, 1.0, opt_cfg.init_lr, opt_cfg.end_lr)
    for w in range(2):
        acc = [torch.zeros_like(p) for p in params]
        for b in batches[2 * w: 2 * w + 2]:
            for p in params:
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(b).loss
            (loss / 2).backward()
            for a, p in zip(acc, params):
                if p.grad is not None:
                    a += p.grad
        for a, p in zip(acc, params):
            p.grad = a
        opt.step(opt_cfg.init_lr * lam(w))
    want = {k: v.detach().clone() for k, v in m.state_dict().items()}
    for k in want:
        assert (got_graph[k].float() - got_eager[k].float()).abs().max().item() < 1e-6, k
        assert (got_graph[k].float() - want[k].float()).abs().max().item() < 1e-5, k
