"""Which CPU ops launch the non-esgpt device kernels of one training step (ATen fills, casts, elementwise, blits):
one eager TrainStep under torch.profiler (with_stack); the CPU op that owns each such kernel (FunctionEvent.kernels)
and the innermost eventstreamgpt_amd frames of its Python stack. Usage: fill_sources.py C4 [graph]"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from eventstreamgpt_amd.data.types import PytorchBatch  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.train import TrainStep  # noqa: E402
from eventstreamgpt_amd.transformer.config import OptimizationConfig  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
bc = CONFIGS[name]
cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
torch.manual_seed(0)
if cfg.structured_event_processing_mode == "nested_attention":
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling as M
else:
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling as M
m = M(cfg).cuda().train()
ts = TrainStep(m, OptimizationConfig(init_lr=1e-3, lr_num_warmup_steps=10, max_training_steps=1000), torch.bfloat16,
               use_graph=graph)
b = bc.batch(0)
hb = PytorchBatch.empty_packed({k: (tuple(v.shape), v.dtype) for k, v in b.as_dict().items()}, pin_memory=True)
hb.copy_(b)
for _ in range(3):
    ts.prefetch(hb)
    ts.step(hb)
ts.check()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    ts.prefetch(hb)
    ts.step(hb)
    torch.cuda.synchronize()
OURS = ("esgpt", "gemm", "attn", "residual", "embed", "bag_", "colsum", "event_stream", "count_k", "reduce_kernel",
        "adamw", "pack_kernel", "seed_bank", "ln_", "bias_act", "na_", "slab_", "zero_kernel", "dq_lead")
cnt = collections.Counter()
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CUDA:
        continue
    for k in getattr(ev, "kernels", []) or []:
        if any(t in k.name for t in OURS):
            continue
        fr = [s for s in (ev.stack or []) if "eventstreamgpt_amd" in s or "tools" in s]
        where = " <- ".join(fr[:3]) if fr else (ev.stack[0] if ev.stack else "?")
        shapes = str(ev.input_shapes)[:60] if ev.input_shapes else ""
        cnt[(k.name[:60], ev.name, shapes, where[:220])] += 1
print(f"{name}: non-esgpt kernels of one {'graph' if graph else 'eager'} step")
for (n, op, shapes, where), c in sorted(cnt.items(), key=lambda x: -x[1]):
    print(f"{c:3d}  {n:60s} {op:24s} {shapes:60s} {where}")
