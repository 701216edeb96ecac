"""Is the C2 step host-bound? Device-resident batches, graph replay; per step: wall time, host time blocked in event
synchronisation (the check_errors hand-off), and host busy time (the rest). FUSE=1: optimizer captured in the step graph; CHECK=0: no error hand-off.
    python tools/host_bound.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.config import OptimizationConfig
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
bc = CONFIGS["C2"]
cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
torch.manual_seed(0)
model = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
fuse = os.environ.get("FUSE", "0") == "1"
ts = TrainStep(model, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=10, max_training_steps=10_000),
               compute_dtype=torch.bfloat16, use_graph=True, fuse_optimizer=fuse,
               check_errors=os.environ.get("CHECK", "1") == "1")
dev_b = [bc.batch(i).packed().to("cuda") for i in range(4)]
blocked = [0.0]
_sync = torch.cuda.Event.synchronize


def timed_sync(self):
    t = time.perf_counter()
    _sync(self)
    blocked[0] += time.perf_counter() - t


torch.cuda.Event.synchronize = timed_sync
for j in range(10):
    ts.step(dev_b[j % 4])
ts.check()
torch.cuda.synchronize()
for rep in range(3):
    blocked[0] = 0.0
    t0 = time.perf_counter()
    for j in range(K):
        ts.step(dev_b[j % 4])
    t_sub = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    print(f"fuse={fuse} check={ts.check_errors} wall {1e3 * t1 / K:.4f} ms/step  submit {1e3 * t_sub / K:.4f}  blocked "
          f"{1e3 * blocked[0] / K:.4f}  busy {1e3 * (t_sub - blocked[0]) / K:.4f}", flush=True)
