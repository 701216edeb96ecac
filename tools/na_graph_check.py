"""TrainStep eager vs HIP-graph for a nested-attention config (default C4 at a small batch), bf16, dropout off:
prints the loss per step and the first step whose device error word is set. ``SPLIT=0`` switches the input
layer to JOINT; ``B`` sets the batch size."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.kernels import check_errors
from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.config import OptimizationConfig
from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

bc = CONFIGS[os.environ.get("CFG", "C4")]
B = int(os.environ.get("B", "4"))
n_steps = 4
batches = [bc.batch(i, batch_size=B, device="cuda").packed() for i in range(n_steps)]


def run(graph: bool):
    kw = dict(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    if os.environ.get("SPLIT", "1") == "0":
        kw["do_split_embeddings"] = False
    cfg = bc.model_config(**kw)
    torch.manual_seed(0)
    m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
    ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=2, max_training_steps=100),
                   torch.bfloat16, use_graph=graph, _force_graph=True)
    out = []
    for i, b in enumerate(batches):
        loss = ts.step(b)
        torch.cuda.synchronize()
        out.append(float(loss))
        try:
            check_errors()
            err = ""
        except ValueError as e:
            err = f"  ERROR: {e}"
        print(f"graph={graph} step {i}: loss {out[-1]:.6f}{err}", flush=True)
        bad_g = [n for n, q in m.named_parameters() if q.grad is not None and not bool(torch.isfinite(q.grad).all())]
        bad_w = [n for n, q in m.named_parameters() if not bool(torch.isfinite(q).all())]
        big = sorted(((float(q.grad.abs().max()), n) for n, q in m.named_parameters() if q.grad is not None),
                     reverse=True)[:3]
        print(f"   nonfinite grads {bad_g[:4]} ({len(bad_g)}), weights {bad_w[:4]} ({len(bad_w)}), max|g| {big}",
              flush=True)
    return out


eager = run(False)
graph = run(os.environ.get("EAGER2") != "1")  # EAGER2=1: eager twice (run-to-run determinism)
print("eager vs graph:", [f"{a - b:.2e}" for a, b in zip(eager, graph)], flush=True)
