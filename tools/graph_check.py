"""Diagnoses HIP-graph capture of the training step stage by stage (forward only, then forward+backward)."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from eventstreamgpt_amd.synthetic import CONFIGS
from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

stage = sys.argv[1] if len(sys.argv) > 1 else "fwd"
bc = CONFIGS["C2"]
cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
torch.manual_seed(0)
m = CIPPTForGenerativeSequenceModeling(cfg).cuda()
batch = bc.batch(0, device="cuda")
eager = m(batch).loss.item()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        out = m(batch)
        if stage == "bwd":
            out.loss.backward()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("warmup ok", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out = m(batch)
    if stage == "bwd":
        out.loss.backward()
torch.cuda.synchronize()
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print(f"replay ok: eager {eager:.6f} graph {out.loss.item():.6f}", flush=True)
