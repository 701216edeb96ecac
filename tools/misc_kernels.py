"""Which host calls launch the small non-esgpt kernels of a C2 step (ATen fills, elementwise, blit copies): one eager
TrainStep under torch.profiler (with_stack); for every device kernel that is not an esgpt kernel, the CPU op that
launched it and the innermost eventstreamgpt_amd / bench frames of that op."""
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
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling  # noqa

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
bc = CONFIGS[name]
cfg = bc.model_config(attention_dropout=0.1, input_dropout=0.1, resid_dropout=0.1)
torch.manual_seed(0)
m = CIPPTForGenerativeSequenceModeling(cfg).cuda().train()
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
cnt = collections.Counter()
for ev in prof.events():
    if ev.device_type != torch.autograd.DeviceType.CUDA:
        continue
    n = ev.name
    if any(t in n for t in ("esgpt", "gemm", "attn", "residual", "embed", "bag_", "colsum", "event_stream", "count_k",
                            "reduce_kernel", "adamw", "pack_kernel", "seed_bank", "ln_", "bias_act", "na_")):
        continue
    parent = ev.cpu_parent
    op = parent.name if parent is not None else "?"
    where = "?"
    if parent is not None and parent.stack:
        fr = [s for s in parent.stack if "eventstreamgpt_amd" in s or "bench" in s or "tools" in s]
        where = " <- ".join(fr[:3]) if fr else parent.stack[0]
    cnt[(n[:70], op, where[:200])] += 1
for (n, op, where), c in sorted(cnt.items(), key=lambda x: -x[1]):
    print(f"{c:3d}  {n:70s} {op:30s} {where}")
