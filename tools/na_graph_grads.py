"""Which gradients differ between the eager and the HIP-graph NA step (C4 config, small batch, bf16, dropout off,
lr ~0 (endless warmup) so both runs see the same weights): prints the parameters with the largest relative gradient difference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.config import OptimizationConfig
from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

bc = CONFIGS["C4"]
batches = [bc.batch(i, batch_size=4, device="cuda").packed() for i in range(3)]


def grads(graph: bool):
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
    ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=int(os.environ.get("WARM", 10**9)),
                                                max_training_steps=10**10),
                   torch.bfloat16, use_graph=graph, _force_graph=True)
    out = []
    for b in batches:
        loss = float(ts.step(b))
        torch.cuda.synchronize()
        out.append((loss, {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None},
                    {n: p.detach().float().clone() for n, p in m.named_parameters()}))
    return out


e, g = grads(False), grads(True)
for step, ((le, ge, pe), (lg, gg, pg)) in enumerate(zip(e, g)):
    diffs = sorted((((ge[k] - gg[k]).abs().max() / ge[k].abs().max().clamp_min(1e-12)).item(), k) for k in ge)[::-1]
    pdiffs = sorted((((pe[k] - pg[k]).abs().max()).item(), k) for k in pe)[::-1]
    print(f"step {step}: loss {le:.6f} vs {lg:.6f}; grad diffs {diffs[:3]}; param diffs after update {pdiffs[:3]}",
          flush=True)
