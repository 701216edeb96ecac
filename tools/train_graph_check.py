"""Checks TrainStep under HIP-graph capture against eager TrainStep (same init, same batches, dropout off), then a
graph run with dropout on. Prints one line per step; any device fault surfaces at the per-step synchronize."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
from eventstreamgpt_amd.transformer.config import OptimizationConfig

bc = CONFIGS[os.environ.get("CFG", "C2")]
n_steps = 4
batches = [bc.batch(i, device="cuda") for i in range(n_steps)]


def run(graph: bool, p: float):
    cfg = bc.model_config(attention_dropout=p, input_dropout=p, resid_dropout=p)
    torch.manual_seed(0)
    m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
    ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=2, max_training_steps=100),
                   torch.bfloat16, use_graph=graph)
    out = []
    for i, b in enumerate(batches):
        loss = ts.step(b)
        torch.cuda.synchronize()
        out.append(float(loss))
        print(f"graph={graph} p={p} step {i}: loss {out[-1]:.6f}", flush=True)
    ts.check()
    return out


eager = run(False, 0.0)
graph = run(True, 0.0)
diff = max(abs(a - b) for a, b in zip(eager, graph))
print(f"eager vs graph max |dloss| = {diff:.3e}", flush=True)
run(True, 0.1)
assert diff < 1e-3, diff
print("ok")
