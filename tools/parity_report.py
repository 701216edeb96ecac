"""Parity diagnostics (GPU): per-tensor gradient errors of the HIP path against the reference goldens (f32) and the
f32 oracle at the C2-C5 widths (bf16 autocast), to size the per-tensor bounds of tests/test_gpu_parity.py.
Error = max |got - want| / max |want| per tensor; also the cosine between the flattened gradients."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import esgpt_oracle as O  # noqa: E402
from helpers import CASES, load_case  # noqa: E402

from eventstreamgpt_amd.synthetic import CONFIGS  # noqa: E402


def _model(cfg):
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    if str(cfg.structured_event_processing_mode) == "conditionally_independent":
        return CIPPTForGenerativeSequenceModeling(cfg)
    return NAPPTForGenerativeSequenceModeling(cfg)


def errs(got: dict, want: dict):
    out = []
    for k, w in want.items():
        g = got.get(k)
        if g is None:
            out.append((float("inf"), 0.0, k))
            continue
        g, w = g.double().cpu().flatten(), w.double().cpu().flatten()
        e = ((g - w).abs().max() / w.abs().max().clamp_min(1e-30)).item()
        cos = torch.nn.functional.cosine_similarity(g, w, dim=0).item() if w.abs().max() > 0 else 1.0
        out.append((e, cos, k))
    return sorted(out, reverse=True)


def golden_f32():
    for name in CASES:
        fx, cfg, batch = load_case(name)
        m = _model(cfg).cuda()
        m.load_state_dict(fx["state_dict"])
        m.train()
        out = m(batch.to("cuda"))
        out.loss.backward()
        got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
        e = errs(got, fx["grads"])
        lrel = abs(out.loss.item() - fx["loss"].item()) / abs(fx["loss"].item())
        print(f"[golden f32] {name}: loss rel {lrel:.2e}; worst grads " +
              ", ".join(f"{k}={x:.2e}" for x, _, k in e[:4]), flush=True)


def width_bf16(name: str, B: int):
    bc = CONFIGS[name]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = _model(cfg).cuda().train()
    batch = bc.batch(0, batch_size=B)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(batch.to("cuda"))
    out.loss.backward()
    got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    trainable = {k for k, p in m.named_parameters() if p.requires_grad}
    p = {k: v.detach().cpu().clone().requires_grad_(k in trainable) for k, v in m.state_dict().items()}
    ref = O.model_losses(p, cfg, batch)
    ref["loss"].backward()
    want = {k: v.grad for k, v in p.items() if v.grad is not None}
    e = errs(got, want)
    lrel = abs(out.loss.item() - ref["loss"].item()) / abs(ref["loss"].item())
    print(f"[bf16 {name} B={B}] loss rel {lrel:.2e}; max grad err {e[0][0]:.2e}; min cos "
          f"{min(c for _, c, _ in e):.6f}; worst " + ", ".join(f"{k}={x:.2e}/{c:.5f}" for x, c, k in e[:5]),
          flush=True)


def width_f32(name: str, B: int):
    bc = CONFIGS[name]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = _model(cfg).cuda().train()
    batch = bc.batch(0, batch_size=B)
    out = m(batch.to("cuda"))
    out.loss.backward()
    got = {k: p.grad for k, p in m.named_parameters() if p.grad is not None}
    trainable = {k for k, p in m.named_parameters() if p.requires_grad}
    p = {k: v.detach().cpu().clone().requires_grad_(k in trainable) for k, v in m.state_dict().items()}
    ref = O.model_losses(p, cfg, batch)
    ref["loss"].backward()
    want = {k: v.grad for k, v in p.items() if v.grad is not None}
    e = errs(got, want)
    lrel = abs(out.loss.item() - ref["loss"].item()) / abs(ref["loss"].item())
    print(f"[f32 {name} B={B}] loss rel {lrel:.2e}; worst grads " + ", ".join(f"{k}={x:.2e}" for x, _, k in e[:5]),
          flush=True)


if __name__ == "__main__":
    torch.set_num_threads(16)
    golden_f32()
    for name, B in (("C2", 4), ("C3", 2), ("C4", 2), ("C5", 2)):
        width_bf16(name, B)
    for name, B in (("C2", 2), ("C3", 1)):
        width_f32(name, B)
