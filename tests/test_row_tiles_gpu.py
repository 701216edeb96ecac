"""Padded-event row blocks in the projection GEMMs (esgpt_row_tiles / esgpt_gemm_row_tiles): the NA dependency-graph
module holds every padded event's G+1 token rows, which the reference compacts away (structured_attention.py:162-165,
186-193). A 64-row block of only padded events' rows skips its k loop in the forward and dX products; every other row
must be bitwise what the unmasked launch computes, and the skipped rows of dX must be exact zeros (their incoming
gradient is zero), so dW — never masked — is unchanged too."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from eventstreamgpt_amd import ops

    return ops.load()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_row_tiles_mask_and_skipped_products(dt):
    from eventstreamgpt_amd.kernels import tickets

    esgpt = _ops()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    n_ev, rpe, D, F = 96, 5, 64, 128  # 480 rows = 7.5 row blocks
    em = torch.rand(n_ev, device=dev, generator=g) > 0.3
    em[40:80] = False  # a run of padded events: rows 200..399 hold whole padded blocks 4 and 5
    tiles = esgpt.row_tiles(em, rpe)
    want = torch.tensor([bool(em[(64 * t) // rpe: min(n_ev, (64 * t + 63) // rpe + 1)].any())
                         for t in range((n_ev * rpe + 63) // 64)], device=dev)
    assert torch.equal(tiles.bool(), want) and not bool(want[4]) and not bool(want[5])
    T = n_ev * rpe
    x = torch.randn(T, D, device=dev, generator=g).to(dt)
    w = torch.randn(F, D, device=dev, generator=g).to(dt) * 0.1
    bias = torch.randn(F, device=dev, generator=g)
    tk = tickets(dev)
    y0 = esgpt.linear(x, w, bias, [], tk)
    y1 = esgpt.linear(x, w, bias, [], tk, tiles)
    rows_on = tiles.bool().repeat_interleave(64)[:T]
    assert torch.equal(y1[rows_on], y0[rows_on])
    assert torch.equal(y1[~rows_on], bias.to(dt).expand(int((~rows_on).sum()), F))  # act(0 + bias)
    # backward: dY zero on the padded events' rows (as the masked module output makes it)
    row_ev = torch.arange(T, device=dev) // rpe
    dy = torch.randn(T, F, device=dev, generator=g).to(dt) * em[row_ev].unsqueeze(1).to(dt)
    dx0, dw0, db0 = esgpt.linear_bwd(dy, x, w, None, -1, None, True, True, tk)
    dx1, dw1, db1 = esgpt.linear_bwd(dy, x, w, None, -1, None, True, True, tk, None, None, None, None, tiles)
    assert torch.equal(dx1[rows_on], dx0[rows_on]) and bool((dx1[~rows_on] == 0).all())
    assert torch.equal(dw1, dw0) and torch.equal(db1, db0)


def test_na_step_with_row_tiles_matches_without():
    """The C4-shaped NA step (dependency graph with padded events): losses and every gradient bitwise equal with the
    row-block skipping on and off."""
    from eventstreamgpt_amd import fused
    from eventstreamgpt_amd.synthetic import CONFIGS
    from eventstreamgpt_amd.transformer.nested_attention_model import NAPPTForGenerativeSequenceModeling

    bc = CONFIGS["C4"]
    cfg = bc.model_config(attention_dropout=0.0, input_dropout=0.0, resid_dropout=0.0)
    torch.manual_seed(0)
    m = NAPPTForGenerativeSequenceModeling(cfg).cuda().train()
    batch = bc.batch(0, batch_size=4, device="cuda")
    assert not bool(batch.event_mask.all())
    real = fused._ops()

    class _NoSkip:  # every row block marked as holding a live event: nothing is skipped
        def __getattr__(self, k):
            if k == "row_tiles":
                return lambda em, rpe: torch.ones((em.numel() * rpe + 63) // 64, dtype=torch.uint8, device=em.device)
            return getattr(real, k)

    saved = fused._ops
    saved_flag = fused.ROW_TILES
    fused.ROW_TILES = True  # (off by default: measured no gain on the C4 step)
    res = {}
    for on in (True, False):
        m.zero_grad(set_to_none=True)
        fused._ops = saved if on else (lambda: _NoSkip())
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(batch)
            out.loss.backward()
        finally:
            fused._ops = saved
            if not on:
                fused.ROW_TILES = saved_flag
        res[on] = (float(out.loss), {k: p.grad.detach().clone() for k, p in m.named_parameters()
                                     if p.grad is not None})
    assert res[True][0] == res[False][0]
    for k, v in res[False][1].items():
        assert torch.equal(res[True][1][k], v), k
