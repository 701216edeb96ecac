"""Eager launches of the C2 output loss (count + event + reduce) for counter collection:
    rocprofv3 --pmc <counters> -- python tools/loss_pmc.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling  # noqa

bc = CONFIGS["C2"]
cfg = bc.model_config()
model = CIPPTForGenerativeSequenceModeling(cfg).cuda()
batch = bc.batch(0, device="cuda")
fwd, nbytes, keep = bench._loss_launcher(model, batch)
for _ in range(5):
    fwd()
torch.cuda.synchronize()
