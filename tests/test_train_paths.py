"""Training-step paths beyond the fused CI graph: the nested-attention step (module path, run eagerly — its PyTorch
GEMMs produced garbage bias gradients under HIP-graph replay) stays finite and matches eager over several optimizer
steps; the CI fused step keeps its graph."""
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
    assert not graph_safe(NAPPTForGenerativeSequenceModeling(na))


@pytest.mark.gpu
def test_nested_attention_train_steps_finite():
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS["C4"]
    batches = [bc.batch(i, batch_size=2, device="cuda").packed() for i in range(4)]
    losses = {}
    for graph in (False, True):
        cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
        torch.manual_seed(0)
        m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
        ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=1, max_training_steps=100),
                       torch.bfloat16, use_graph=graph)
        assert ts.use_graph is False
        losses[graph] = [float(ts.step(b)) for b in batches]
        ts.check()
        assert all(torch.isfinite(p).all() for p in m.parameters())
    assert all(abs(a - b) < 1e-4 * max(1.0, abs(a)) for a, b in zip(losses[False], losses[True]))


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
