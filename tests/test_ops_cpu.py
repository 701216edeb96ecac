"""CPU checks of the custom-operator layer (``torch.ops.esgpt``, csrc/torch_ops.cpp + eventstreamgpt_amd/ops.py):
the library loads, every operator has a schema, the fake (meta) kernels give the HIP kernels' output shapes, the
registered autograd formulas run end to end on meta tensors (shapes / which inputs get gradients), and there is no
CPU kernel (no silent fallback)."""
import os

import pytest
import torch

from eventstreamgpt_amd import ops as O

pytestmark = pytest.mark.skipif(not os.path.exists(O.TORCH_LIB_PATH), reason="libesgpt_torch.so not built")
M = "meta"


@pytest.fixture(scope="module")
def esgpt():
    return O.load()


def test_every_operator_has_a_schema(esgpt):
    for name in O.OPS:
        op = getattr(esgpt, name)
        assert op.default._schema.name == f"esgpt::{name}"


def _batch(B=2, L=5, Mx=3, S=2, dev=M):
    return (torch.empty(B, L, dtype=torch.bool, device=dev), torch.empty(B, L, device=dev), None,
            torch.empty(B, L, Mx, dtype=torch.long, device=dev), torch.empty(B, L, Mx, dtype=torch.long, device=dev),
            torch.empty(B, L, Mx, device=dev), torch.empty(B, L, Mx, dtype=torch.bool, device=dev),
            torch.empty(B, S, dtype=torch.long, device=dev), torch.empty(B, S, dtype=torch.long, device=dev))


def _err(dev=M):
    return torch.empty(2, dtype=torch.long, device=dev)


def _tk(dev=M):
    return torch.empty(64, dtype=torch.int32, device=dev)


def test_embed_joint_fake_and_autograd(esgpt):
    table = torch.empty(11, 8, device=M, requires_grad=True)
    out = esgpt.embed_joint(table, *_batch(), [], None, None, 2, 0.5, 0.5, 1, _err())
    assert out.shape == (2, 5, 1, 8) and out.dtype == torch.float32
    out.sum().backward()
    assert table.grad.shape == (11, 8)


def test_embed_split_bags_fake_and_autograd(esgpt):
    ct = torch.empty(11, 4, device=M, requires_grad=True)
    nt = torch.empty(11, 6, device=M, requires_grad=True)
    buckets = [3] + [1, 2, 4] + [0] * 5 + [0, 2, 4] + [0] * 5
    x = esgpt.embed_split_bags(ct, nt, *_batch(), buckets, 0, 0.5, 0.5, 0.0, 3, _err())
    assert x.shape == (2 * 5 * 3, 10)
    x.sum().backward()
    assert ct.grad.shape == (11, 4) and nt.grad.shape == (11, 6)


def test_embed_epilogue_autograd(esgpt):
    y = torch.empty(2 * 5 * 3, 8, device=M, requires_grad=True)
    out = esgpt.embed_epilogue(y, *_batch(), 3, 8, None, None)
    assert out.shape == (2, 5, 3, 8)
    out.sum().backward()
    assert y.grad.shape == y.shape


@pytest.mark.parametrize("skf", [False, True])
def test_attention_fake_and_autograd(esgpt, skf):
    qkv = torch.empty(3, 7, 3 * 32, dtype=torch.bfloat16, device=M, requires_grad=True)
    o, lse, keep = esgpt.attention(qkv, None, None, 4, 0, skf, 0.0, None)
    assert o.shape == (3, 7 - skf, 32) and o.dtype == torch.bfloat16 and lse.shape == (3, 4, 7 - skf)
    o.float().sum().backward()
    assert qkv.grad.shape == qkv.shape


def test_residual_ln_autograd(esgpt):
    x = torch.empty(6, 16, device=M, requires_grad=True)
    y = torch.empty(6, 16, dtype=torch.bfloat16, device=M, requires_grad=True)
    b, w, lb = (torch.empty(16, device=M, requires_grad=True) for _ in range(3))
    h, out, mean, rstd = esgpt.residual_ln(x, y, b, w, lb, None, 0.0, None, 1e-5, torch.bfloat16)
    assert h.dtype == torch.float32 and out.dtype == torch.bfloat16 and mean.shape == (6,)
    (h.sum() + out.float().sum()).backward()
    for t in (x, y, b, w, lb):
        assert t.grad is not None and t.grad.shape == t.shape, t.shape
    # only `out` used: dh is not materialised
    x2 = torch.empty(6, 16, device=M, requires_grad=True)
    _, out2, _, _ = esgpt.residual_ln(x2, None, None, w, lb, None, 0.0, None, 1e-5, torch.float32)
    out2.sum().backward()
    assert x2.grad.shape == (6, 16)


def test_linear_and_mlp_autograd_route_f32_master_gradients(esgpt):
    x = torch.empty(16, 8, dtype=torch.bfloat16, device=M, requires_grad=True)
    masters = [torch.empty(n, 8, device=M, requires_grad=True) for n in (8, 8, 16)]
    w_lp = torch.empty(32, 8, dtype=torch.bfloat16, device=M)
    bias = torch.empty(32, device=M, requires_grad=True)
    y = esgpt.linear(x, w_lp, bias, masters, _tk())
    assert y.shape == (16, 32)
    y.float().sum().backward()
    assert x.grad.dtype == torch.bfloat16 and bias.grad.shape == (32,)
    for m in masters:
        assert m.grad.dtype == torch.float32 and m.grad.shape == m.shape
    pf, pp = torch.empty(24, 8, device=M, requires_grad=True), torch.empty(8, 24, device=M, requires_grad=True)
    bf = torch.empty(24, device=M, requires_grad=True)
    x3 = torch.empty(16, 8, dtype=torch.bfloat16, device=M, requires_grad=True)
    bp = torch.empty(8, device=M, requires_grad=True)
    y3, pre, g = esgpt.mlp(x3, pf.bfloat16(), pp.bfloat16(), bf, bp, 0, pf, pp, _tk())
    assert y3.shape == (16, 8) and pre.shape == g.shape == (16, 24)
    y3.float().sum().backward()
    assert pf.grad.shape == pf.shape and pp.grad.shape == pp.shape and bf.grad.shape == (24,) and x3.grad is not None
    assert bp.grad.shape == (8,)


def test_head_loss_and_output_loss_autograd(esgpt):
    from eventstreamgpt_amd import _lib as L

    terms = [L.TERM_SINGLE, 1, 1, 4, 1, 10, 0, 0]
    xc = torch.empty(10, 8, dtype=torch.bfloat16, device=M, requires_grad=True)
    cw = [torch.empty(11, 8, device=M, requires_grad=True), torch.empty(2, 8, device=M, requires_grad=True)]
    cb = [torch.empty(11, device=M, requires_grad=True), torch.empty(2, device=M, requires_grad=True)]
    wc = torch.empty(16, 8, dtype=torch.bfloat16, device=M)
    bc = torch.empty(16, device=M)
    losses, dzc, dzt, dbias = esgpt.head_loss(xc, None, *_batch(), terms, [1, 1, 13], [0.0, 1.0], 1, 1, wc, bc, None,
                                              None, cw, cb, [], [], _err(), _tk(), None)
    assert losses.shape == (3,) and dzc.shape == (10, 16) and dbias.shape == (2, 16)
    losses[-1].backward()
    assert xc.grad.shape == xc.shape and all(p.grad is not None for p in cw + cb)
    zc = torch.empty(10, 16, dtype=torch.bfloat16, device=M, requires_grad=True)
    zb = torch.empty(16, dtype=torch.bfloat16, device=M, requires_grad=True)
    out = esgpt.output_loss(zc, None, zb, *_batch(), 1, 1, terms, [1, 1, 13], [0.0, 1.0], _err())
    out[0][-1].backward()
    assert zc.grad.shape == zc.shape and zb.grad.shape == zb.shape


def test_no_cpu_kernel(esgpt):
    qkv = torch.zeros(1, 4, 3 * 8)
    with pytest.raises(NotImplementedError):
        esgpt.attention(qkv, None, None, 1, 0, False, 0.0, None)
