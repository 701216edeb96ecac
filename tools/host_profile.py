"""Host-side cost of the training step (is the step host-bound?): builds the bench's C2 TrainStep, warms up, then
times the submission of K steps (no sync inside) against the device time of the same K steps, and runs cProfile
over the submissions.
    python tools/host_profile.py [config] [steps]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.data.types import PytorchBatch
from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.train import TrainStep
from eventstreamgpt_amd.transformer.config import OptimizationConfig

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
bc = CONFIGS[name]
cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
torch.manual_seed(0)
if cfg.structured_event_processing_mode == "conditionally_independent":
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling as M
else:
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling as M
model = M(cfg).cuda().train()
ts = TrainStep(model, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=10, max_training_steps=10_000),
               compute_dtype=torch.bfloat16, use_graph=True)
host = []
for i in range(4):
    b = bc.batch(i)
    hb = PytorchBatch.empty_packed({k: (tuple(v.shape), v.dtype) for k, v in b.as_dict().items()}, pin_memory=True)
    hb.copy_(b)
    host.append(hb)


PREFETCH = os.environ.get("PREFETCH", "1") == "1"


def run(n, j0):
    for j in range(j0, j0 + n):
        ts.step(host[j % 4])
        if PREFETCH:
            ts.prefetch(host[(j + 1) % 4])


print(f"prefetch={PREFETCH}")
if PREFETCH:
    ts.prefetch(host[0])
run(8, 0)
ts.check()
torch.cuda.synchronize()
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    run(K, 8)
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name} rep {rep}: host submit {1e3 * (t1 - t0) / K:.3f} ms/step, wall {1e3 * (t2 - t0) / K:.3f} ms/step, "
          f"device span {e0.elapsed_time(e1) / K:.3f} ms/step", flush=True)
ts.check()
# the pieces of one submission
segs = next(v for v in ts.graphs.values() if v is not None)[0]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    for g, _ in segs:
        g.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"graph replay alone: host {1e3 * (t1 - t0) / K:.3f} ms/replay, wall {1e3 * (t2 - t0) / K:.3f} ms/replay",
      flush=True)
if os.environ.get("CPROFILE", "1") != "1":
    sys.exit(0)
pr = cProfile.Profile()
pr.enable()
run(K, 8)
pr.disable()
torch.cuda.synchronize()
ts.check()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
