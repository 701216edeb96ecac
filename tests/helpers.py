"""Shared test helpers: loading golden fixtures (weights_only) and building configs from them."""
import json
import os

import torch

from eventstreamgpt_amd.data.types import PytorchBatch
from eventstreamgpt_amd.transformer.config import StructuredTransformerConfig

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["ci_small", "ci_lnm_norm", "ci_split", "na_small", "na_joint_attn"]


def load_case(name):
    fx = torch.load(os.path.join(GOLDEN, f"{name}.pt"), weights_only=True)
    kw = json.loads(fx["config_kwargs"])
    cfg = StructuredTransformerConfig(**kw)
    batch = PytorchBatch(**fx["batch"])
    return fx, cfg, batch


def rel_err(a, b):
    a = a.double()
    b = b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()
