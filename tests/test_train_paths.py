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
