"""The two loss event kernels (csrc/losses.hip) on identical inputs: the row-staged kernel (whole logit row in LDS,
complete gradient rows stored, no zero-fill) and the generic column-by-column kernel (ESGPT_LOSS_ROW_STAGE=0,
taken for rows too wide for LDS). Both restate model_output.py:1311-1721 with the same per-term math, so the losses
and every parameter gradient must be bitwise equal — CI (shifted content head with the TTE columns in the same row
and the bias row) and NA (per-level rows, separate TTE head), f32 and bf16. Oracle parity of the default path is
in test_gpu_parity.py."""
import os

import pytest
import torch

from eventstreamgpt_amd.synthetic import CONFIGS

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(cfg_name: str, B: int, dtype, stage: str):
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS[cfg_name]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    ci = str(cfg.structured_event_processing_mode) == "conditionally_independent"
    m = (CIPPTForGenerativeSequenceModeling if ci else NAPPTForGenerativeSequenceModeling)(cfg).to(DEV).train()
    batch = bc.batch(0, batch_size=B).to(DEV)
    old = os.environ.get("ESGPT_LOSS_ROW_STAGE")
    os.environ["ESGPT_LOSS_ROW_STAGE"] = stage
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
            out = m(batch)
        out.loss.backward()
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["ESGPT_LOSS_ROW_STAGE"]
        else:
            os.environ["ESGPT_LOSS_ROW_STAGE"] = old
    return out.loss.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("cfg_name,B,dtype", [("C2", 4, torch.bfloat16), ("C2", 2, torch.float32),
                                              ("C4", 2, torch.bfloat16), ("C1", 4, torch.float32)])
def test_row_staged_loss_kernel_equals_generic(cfg_name, B, dtype):
    from eventstreamgpt_amd.kernels import check_errors

    l1, g1 = _run(cfg_name, B, dtype, "1")
    l0, g0 = _run(cfg_name, B, dtype, "0")
    check_errors()
    assert torch.equal(l1, l0), (l1.item(), l0.item())
    assert g1.keys() == g0.keys()
    bad = [k for k in g1 if not torch.equal(g1[k], g0[k])]
    assert not bad, bad[:5]
