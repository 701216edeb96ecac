"""The three loss event kernels of csrc/losses.hip on identical inputs, through ``esgpt::output_loss``'s explicit
``path`` argument (esgpt_output_loss_ex): STREAM (default; the row streamed once in 16-B chunks, dense per-range
rules + sparse patches), ROW_STAGED (the whole row in LDS) and GENERIC (column by column over zero-filled
gradients). All restate model_output.py:1311-1721 with the same per-element formulas, so every logit gradient and
the position-0 bias rows must be bitwise equal. The per-term losses of ROW_STAGED and GENERIC are bitwise equal
(per-row contributions, same order); STREAM sums its multi-label BCE columns in another order and its contributions
per workgroup of four rows, so its losses agree to f32 rounding (checked at 1e-5 relative). Layouts: CI (shifted content
head with the TTE columns in the same row and the bias row) at the C1 / C2 / C5 widths (C5: V = 10,210, LNM K = 8,
M = 32) and NA (per-level rows, separate TTE head) at C4, f32 and bf16. Oracle parity of the default path through
the full models is in test_gpu_parity.py."""
import pytest
import torch

from eventstreamgpt_amd import _lib as L
from eventstreamgpt_amd.kernels import batch_args, err_word, terms_list, tte_lists
from eventstreamgpt_amd.synthetic import CONFIGS

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _layout(cfg_name):
    from eventstreamgpt_amd.transformer import model_output as MO
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS[cfg_name]
    cfg = bc.model_config()
    ci = str(cfg.structured_event_processing_mode) == "conditionally_independent"
    m = (CIPPTForGenerativeSequenceModeling if ci else NAPPTForGenerativeSequenceModeling)(cfg)
    layer = m.output_layer
    layer._layout = layer._build_layout()
    cls_all, reg_all = MO.all_classification_measurements(layer), MO.all_regression_measurements(cfg)
    if ci:
        terms, _ = layer._terms_for(cls_all, reg_all, 0)
        tte = layer._tte_spec(layer._layout["n_content"])
        n_cols = layer._layout["n_content"] + (1 if tte.kind == L.TTE_EXP else 3 * tte.K)
        return bc, terms, tte, 1, 1, n_cols, None
    G = len(cfg.measurements_per_dep_graph_level)
    terms = []
    for i in range(1, G):
        cat, num = MO._level_sets(cfg.measurements_per_dep_graph_level[i])
        t, _ = layer._terms_for(cat & cls_all, num & reg_all, i - 1)
        terms += t
    tte = layer._tte_spec(0)
    return bc, terms, tte, 0, G - 1, layer._layout["n_content"], 1 if tte.kind == L.TTE_EXP else 3 * tte.K


def _run(esgpt, cfg_name, B, dtype, path, seed=5):
    bc, terms, tte, shift, n_levels, n_cols, n_tte = _layout(cfg_name)
    b = bc.batch(1, batch_size=B, device=DEV)
    C = (n_cols + 7) // 8 * 8
    g = torch.Generator(device=DEV).manual_seed(seed)
    Lq = b.dynamic_indices.shape[1]
    zc = (2 * torch.randn(B * Lq * n_levels, C, device=DEV, generator=g)).to(dtype)
    zt = None if n_tte is None else torch.randn(B * Lq, n_tte, device=DEV, generator=g).to(dtype)
    bias = torch.randn(C, device=DEV, generator=g).to(dtype) if shift else None
    err = err_word(torch.device(DEV))
    ti, tf = tte_lists(tte)
    out = esgpt.output_loss(zc, zt, bias, *batch_args(b), n_levels, shift, terms_list(terms), ti, tf, err, path)
    torch.cuda.synchronize()
    assert int(err[0]) == 0
    return out, terms


CASES = [("C1", 4, torch.float32), ("C2", 4, torch.bfloat16), ("C2", 2, torch.float32), ("C4", 2, torch.bfloat16),
         ("C4", 2, torch.float32), ("C5", 2, torch.bfloat16)]


@pytest.mark.parametrize("cfg_name,B,dtype", CASES)
def test_loss_paths_equal(cfg_name, B, dtype):
    from eventstreamgpt_amd import ops

    esgpt = ops.load()
    (l_g, dzc_g, dzt_g, db_g), terms = _run(esgpt, cfg_name, B, dtype, L.LOSS_PATH_GENERIC)
    paths = [L.LOSS_PATH_STREAM, L.LOSS_PATH_AUTO]
    esz = 2 if dtype == torch.bfloat16 else 4
    if _layout(cfg_name)[5] * (esz + 4) <= 64 * 1024:
        paths.append(L.LOSS_PATH_ROW_STAGED)
    for path in paths:
        (l, dzc, dzt, db), _ = _run(esgpt, cfg_name, B, dtype, path)
        assert torch.equal(dzc, dzc_g), (path, float((dzc.float() - dzc_g.float()).abs().max()))
        assert torch.equal(dzt, dzt_g) and torch.equal(db, db_g), path
        for i in range(l.numel()):
            assert abs(float(l[i]) - float(l_g[i])) <= 1e-5 * max(1.0, abs(float(l_g[i]))), (path, i)
        if path == L.LOSS_PATH_ROW_STAGED:
            assert torch.equal(l, l_g)


def test_forced_path_that_does_not_apply_is_refused():
    """ROW_STAGED on a row too wide for LDS (f32 C5 logits: 10,640 × 8 B per wave) raises instead of falling back."""
    from eventstreamgpt_amd import ops

    esgpt = ops.load()
    with pytest.raises(RuntimeError):
        _run(esgpt, "C5", 1, torch.float32, L.LOSS_PATH_ROW_STAGED)
