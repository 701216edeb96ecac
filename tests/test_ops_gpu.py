"""The custom operators (torch.ops.esgpt) against the raw C ABI (ctypes, exactly the reference-side binding of
INTEGRATION.md) on the same inputs: identical results, bit for bit (every kernel, the embedding-bag backward
included, sums in a fixed order)."""
import ctypes

import pytest
import torch

from eventstreamgpt_amd import _lib as L
from eventstreamgpt_amd.kernels import BatchView, batch_args, err_word, tickets
from eventstreamgpt_amd.synthetic import CONFIGS

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def env():
    from eventstreamgpt_amd import ops

    return ops.load(), L.load()


def _g(seed):
    return torch.Generator(device=DEV).manual_seed(seed)


def test_attention_fwd_bwd_equal_c_abi(env):
    esgpt, lib = env
    B, T, H, hd = 3, 200, 4, 64
    D = H * hd
    qkv = (0.5 * torch.randn(B, T, 3 * D, device=DEV, generator=_g(0))).bfloat16()
    km = torch.rand(B, T, device=DEV, generator=_g(1)) > 0.1
    o, lse, keep = esgpt.attention(qkv, km, km, H, 0, False, 0.0, None)
    o2 = torch.empty_like(o)
    lse2 = torch.empty_like(lse)
    base, es = qkv.data_ptr(), 2
    L.check(lib.esgpt_attn_fwd(base, base + D * es, base + 2 * D * es, 3 * D, T, o2.data_ptr(), D, lse2.data_ptr(),
                               km.data_ptr(), km.data_ptr(), B, H, T, T, hd, 0, 0.0, None, L.BF16, L.stream()), "fwd")
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    do = torch.randn(B, T, D, device=DEV, generator=_g(2)).bfloat16()
    t = tickets(torch.device(DEV))
    dqkv = esgpt.attention_bwd(qkv, o, do, lse, km, km, H, 0, False, 0.0, None, keep, t)
    d2 = torch.empty_like(qkv)
    nb = lib.esgpt_attn_bwd_workspace(B, H, T, T, hd)
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=DEV)
    db = d2.data_ptr()
    cnt = t.data_ptr() if lib.esgpt_attn_bwd_counters(B, H, T) <= t.numel() else None
    L.check(lib.esgpt_attn_bwd(base, base + D * es, base + 2 * D * es, 3 * D, T, o.data_ptr(), D, do.data_ptr(), D,
                               lse.data_ptr(), km.data_ptr(), km.data_ptr(), db, db + D * es, db + 2 * D * es, 3 * D,
                               B, H, T, T, hd, 0, 0.0, None, L.BF16, ws.data_ptr(), nb, cnt, L.stream()), "bwd")
    assert torch.equal(dqkv, d2)


@pytest.mark.parametrize("hd,T,window", [(64, 256, 0), (64, 200, 0), (16, 256, 0), (32, 300, 32), (128, 100, 0),
                                          (64, 600, 0)])
def test_attention_keep_bits_equal_rehash(env, hd, T, window):
    """With dropout, the operator's backward reads the keep bits its forward wrote (esgpt_attn_fwd_ex /
    esgpt_attn_bwd_ex); the plain C ABI backward regenerates the mask from the seed. Both must give the same dqkv
    bit for bit (same mask), including padded keys / queries, local windows, several key blocks and hd 16 / 128."""
    esgpt, lib = env
    B, H = 2, 4
    D = H * hd
    qkv = (0.5 * torch.randn(B, T, 3 * D, device=DEV, generator=_g(10))).bfloat16()
    km = torch.rand(B, T, device=DEV, generator=_g(11)) > 0.1
    seed = torch.tensor([987654321], dtype=torch.int64, device=DEV)
    o, lse, keep = esgpt.attention(qkv, km, km, H, window, False, 0.1, seed)
    assert keep.numel() == B * H * T * ((T + 31) // 32)
    do = torch.randn(B, T, D, device=DEV, generator=_g(12)).bfloat16()
    t = tickets(torch.device(DEV))
    d_bits = esgpt.attention_bwd(qkv, o, do, lse, km, km, H, window, False, 0.1, seed, keep, t)
    d_hash = esgpt.attention_bwd(qkv, o, do, lse, km, km, H, window, False, 0.1, seed, None, t)
    assert torch.isfinite(d_bits.float()).all()
    assert torch.equal(d_bits, d_hash)
    # and the plain forward entry point draws the same output
    o2, lse2 = torch.empty_like(o), torch.empty_like(lse)
    base, es = qkv.data_ptr(), 2
    L.check(lib.esgpt_attn_fwd(base, base + D * es, base + 2 * D * es, 3 * D, T, o2.data_ptr(), D, lse2.data_ptr(),
                               km.data_ptr(), km.data_ptr(), B, H, T, T, hd, window, 0.1, seed.data_ptr(), L.BF16,
                               L.stream()), "fwd")
    assert torch.equal(o, o2) and torch.equal(lse, lse2)


def test_embed_joint_and_bag_bwd_equal_c_abi(env):
    esgpt, lib = env
    bc = CONFIGS["C2"]
    b = bc.batch(0, batch_size=8, device=DEV)
    V, Dm = 1210, 256
    table = torch.randn(V, Dm, device=DEV, generator=_g(3))
    err = err_word(torch.device(DEV))
    out = esgpt.embed_joint(table, *batch_args(b), [], None, None, L.EMB_STATIC, 0.5, 0.5, 1, err)
    bv = BatchView(b)
    out2 = torch.empty_like(out)
    L.check(lib.esgpt_embed_joint_fwd(bv.ref, None, table.data_ptr(), V, Dm, None, None, L.EMB_STATIC, 0.5, 0.5,
                                      out2.data_ptr(), err.data_ptr(), L.stream()), "embed")
    assert torch.equal(out, out2)
    dsrc = torch.randn(8 * bc.seq_len, Dm, device=DEV, generator=_g(4))
    dt = esgpt.embed_bag_bwd(dsrc, *batch_args(b), [], L.BAG_JOINT, L.EMB_STATIC, 0.5, 0.5, Dm, Dm, V, 1)
    dt2 = torch.empty_like(dt)
    nb = lib.esgpt_embed_bag_bwd_workspace(bv.ref, 1, V, Dm)
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=DEV)
    L.check(lib.esgpt_embed_bag_bwd(bv.ref, None, L.BAG_JOINT, L.EMB_STATIC, 0.5, 0.5, dsrc.data_ptr(), Dm, Dm, V,
                                    dt2.data_ptr(), ws.data_ptr(), nb, L.stream()), "bag_bwd")
    assert torch.equal(dt, dt2)


def test_output_loss_equal_c_abi(env):
    esgpt, lib = env
    from eventstreamgpt_amd.kernels import terms_list, tte_lists
    from eventstreamgpt_amd.transformer import model_output as MO
    from eventstreamgpt_amd.transformer.conditionally_independent_model import CIPPTForGenerativeSequenceModeling

    bc = CONFIGS["C2"]
    m = CIPPTForGenerativeSequenceModeling(bc.model_config())
    layer = m.output_layer
    layer._layout = layer._build_layout()
    terms, _ = layer._terms_for(MO.all_classification_measurements(layer), MO.all_regression_measurements(m.config), 0)
    tte = layer._tte_spec(layer._layout["n_content"])
    b = bc.batch(1, batch_size=8, device=DEV)
    C = 1624
    zc = torch.randn(8 * bc.seq_len, C, device=DEV, generator=_g(5)).bfloat16()
    bias = torch.randn(C, device=DEV, generator=_g(6)).bfloat16()
    err = err_word(torch.device(DEV))
    ti, tf = tte_lists(tte)
    losses, dzc, _, dbias = esgpt.output_loss(zc, None, bias, *batch_args(b), 1, 1, terms_list(terms), ti, tf, err)
    bv = BatchView(b)
    arr = (L.EsgptLossTerm * len(terms))(*terms)
    l2, d2, db2 = torch.empty_like(losses), torch.empty_like(dzc), torch.empty_like(dbias)
    nb = lib.esgpt_output_loss_workspace(8, bc.seq_len, len(terms))
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=DEV)
    L.check(lib.esgpt_output_loss(bv.ref, zc.data_ptr(), C, 1, 1, bias.data_ptr(), zc.data_ptr(), C, L.BF16, arr,
                                  len(terms), ctypes.byref(tte), d2.data_ptr(), d2.data_ptr(), db2.data_ptr(),
                                  l2.data_ptr(), ws.data_ptr(), nb, err.data_ptr(), L.stream()), "loss")
    assert torch.equal(losses, l2) and torch.equal(dzc, d2) and torch.equal(dbias, db2)


def test_linear_and_residual_ln_equal_c_abi(env):
    esgpt, lib = env
    T, din, dout = 1024, 256, 1024
    x = torch.randn(T, din, device=DEV, generator=_g(7)).bfloat16()
    w = (0.05 * torch.randn(dout, din, device=DEV, generator=_g(8))).bfloat16()
    b = torch.randn(dout, device=DEV, generator=_g(9))
    pre, y = esgpt.linear_act(x, w, b, 0)
    pre2, y2 = torch.empty_like(pre), torch.empty_like(y)
    L.check(lib.esgpt_linear_fwd(x.data_ptr(), din, w.data_ptr(), T, din, dout, b.data_ptr(), 0, pre2.data_ptr(),
                                 y2.data_ptr(), dout, L.stream()), "linear_fwd")
    assert torch.equal(pre, pre2) and torch.equal(y, y2)
    dy = torch.randn(T, dout, device=DEV, generator=_g(10)).bfloat16()
    t = tickets(torch.device(DEV))
    dx, dw, db = esgpt.linear_bwd(dy, x, w, None, -1, None, True, True, t)
    dx2, dw2, db2 = torch.empty_like(dx), torch.empty_like(dw), torch.empty_like(db)
    nb = lib.esgpt_linear_bwd_workspace(T, din, dout, 1)
    ws = torch.empty(max(1, nb), dtype=torch.uint8, device=DEV)
    L.check(lib.esgpt_linear_bwd(dy.data_ptr(), dout, x.data_ptr(), din, w.data_ptr(), T, din, dout, None, -1, None,
                                 0, dx2.data_ptr(), din, dw2.data_ptr(), db2.data_ptr(), ws.data_ptr(), nb,
                                 t.data_ptr(), L.stream()), "linear_bwd")
    assert torch.equal(dx, dx2) and torch.equal(dw, dw2) and torch.equal(db, db2)
    N, D = 600, 256
    h0 = torch.randn(N, D, device=DEV, generator=_g(11))
    yy = torch.randn(N, D, device=DEV, generator=_g(12)).bfloat16()
    lw, lb, bb = (torch.randn(D, device=DEV, generator=_g(13 + i)) for i in range(3))
    h, out, mean, rstd = esgpt.residual_ln(h0, yy, bb, lw, lb, None, 0.0, None, 1e-5, torch.bfloat16)
    h2, out2, m2, r2 = torch.empty_like(h), torch.empty_like(out), torch.empty_like(mean), torch.empty_like(rstd)
    L.check(lib.esgpt_residual_ln_fwd(h0.data_ptr(), yy.data_ptr(), L.BF16, bb.data_ptr(), None, 0.0, None,
                                      lw.data_ptr(), lb.data_ptr(), 1e-5, N, D, h2.data_ptr(), out2.data_ptr(), L.BF16,
                                      m2.data_ptr(), r2.data_ptr(), L.stream()), "ln_fwd")
    assert torch.equal(h, h2) and torch.equal(out, out2) and torch.equal(mean, m2) and torch.equal(rstd, r2)


def test_adamw_op_equals_c_abi(env):
    esgpt, lib = env
    from eventstreamgpt_amd.train import FusedAdamW

    g = torch.Generator().manual_seed(0)
    base = [torch.randn(s, generator=g) for s in [(300, 64), (7,), (4099,)]]
    grads = [torch.randn(b.shape, generator=g).to(DEV) for b in base]
    pa = [b.clone().to(DEV).requires_grad_(True) for b in base]
    pb = [b.clone().to(DEV).requires_grad_(True) for b in base]
    oa, ob = FusedAdamW(pa, lr=1e-2), FusedAdamW(pb, lr=1e-2)
    for p, gr in zip(pa, grads):
        p.grad = gr.clone()
    for p, gr in zip(pb, grads):
        p.grad = gr.clone()
    import ctypes

    for _ in range(2):
        oa.step()  # torch.ops.esgpt.adamw_dev: esgpt_adamw_prepare + esgpt_adamw_dev
        plan = ob._plan()
        sc = L.EsgptLrSchedule(0, 0, 1, 1.0, 1e-2, 0.0)
        L.check(lib.esgpt_adamw_prepare(ob._counters.data_ptr(), plan["active_dev"].data_ptr(), len(plan["active"]),
                                        len(pb), ctypes.byref(sc), 0.9, 0.999, plan["per"].data_ptr(),
                                        ob._lr_dev.data_ptr(), None, L.stream()), "adamw_prepare")
        L.check(lib.esgpt_adamw_dev(plan["table"].data_ptr(), plan["blocks"].data_ptr(), plan["blocks"].numel(),
                                    ob._lr_dev.data_ptr(), 0.9, 0.999, 1e-8, 0.01, plan["per"].data_ptr(), None,
                                    L.stream()), "adamw_dev")
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)
    assert torch.equal(oa._counters, ob._counters) and oa._counters.tolist() == [2, 2, 2, 2]  # + the schedule's step


def test_pack_equals_cat_cast_and_c_abi(env):
    """esgpt::pack (one launch) = torch.cat + zero tail + cast, bit for bit (bf16 round-to-nearest-even), over
    more segments than one launch carries (48), odd lengths and unaligned starts; and = the raw C ABI."""
    esgpt, lib = env
    g = _g(21)
    ts = [torch.randn(n, device=DEV, generator=g) * 3 for n in [5, 256 * 7, 1, 2049, 64, 3] * 9]  # 54 segments
    ts[7][0] = float("nan")
    groups, tails, codes = [30, 24, 24], [13, 0, 5], [L.BF16, L.F32, L.BF16]
    srcs = ts[:30] + ts[30:] + ts[30:]
    out = esgpt.pack(srcs, groups, tails, codes)
    k = 0
    for o, n_src, tail, code in zip(out, groups, tails, codes):
        ref = torch.cat([t.reshape(-1) for t in srcs[k: k + n_src]] + [torch.zeros(tail, device=DEV)])
        k += n_src
        ref = ref.to(torch.bfloat16 if code == L.BF16 else torch.float32)
        assert o.dtype == ref.dtype and o.shape == ref.shape
        assert torch.equal(o.view(torch.int16) if code == L.BF16 else o.view(torch.int32),
                           ref.view(torch.int16) if code == L.BF16 else ref.view(torch.int32))
    # raw C ABI: the first group's segments, the tail on the last one
    dst = torch.full((out[0].numel(),), 7.0, device=DEV).bfloat16()
    segs, off = [], 0
    for j, t in enumerate(srcs[:30]):
        n = t.numel()
        segs.append(L.EsgptPackSeg(t.data_ptr(), dst.data_ptr() + 2 * off, n, n + (13 if j == 29 else 0), L.BF16, 0))
        off += n
    arr = (L.EsgptPackSeg * len(segs))(*segs)
    L.check(lib.esgpt_pack(arr, len(segs), L.stream()), "pack")
    assert torch.equal(dst.view(torch.int16), out[0].view(torch.int16))


def test_linear_bwd_row_sum_addend(env):
    """esgpt_linear_bwd_ex's db_extra: db = alpha·(Σ_rows dy + Σ_b extra[b]) in the same launch (the head's
    position-0 bias rows), for a split-K plan and a whole-K plan; dx / dw unchanged."""
    esgpt, _ = env
    t = tickets(torch.device(DEV))
    for T, din, dout in [(8192, 256, 1624), (256, 64, 24)]:
        x = torch.randn(T, din, device=DEV, generator=_g(31)).bfloat16()
        w = (0.05 * torch.randn(dout, din, device=DEV, generator=_g(32))).bfloat16()
        dy = torch.randn(T, dout, device=DEV, generator=_g(33)).bfloat16()
        extra = torch.randn(32, dout, device=DEV, generator=_g(34))
        alpha = torch.tensor([0.75], device=DEV)
        dx, dw, db = esgpt.linear_bwd(dy, x, w, alpha, -1, None, True, True, t)
        dx2, dw2, db2 = esgpt.linear_bwd(dy, x, w, alpha, -1, None, True, True, t, extra)
        assert torch.equal(dx, dx2) and torch.equal(dw, dw2)
        ref = db.double() + extra.double().sum(0) * 0.75
        assert float((db2.double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max()), (T, din, dout)


def test_linear_bwd_split_streams_equal_grouped(env):
    """esgpt_linear_bwd_split (dX on the current stream, dW / db on the weight-gradient stream, joined by
    esgpt::weight_grad_join) equals the grouped one-launch backward bit for bit: same tiles, same split plan — for
    the step's projection shapes (split-K dW, the 128x128 head dW), the activation-gradient epilogue, alpha, the
    bias-row addend and a dW-only call; the operand memory is held for the side stream while the current stream
    allocates and overwrites in between."""
    esgpt, _ = env
    dev = torch.device(DEV)
    t0, t1 = tickets(dev), tickets(dev, 1)
    cases = [(8192, 256, 1024, 0, True), (8192, 1024, 256, -1, True), (8192, 256, 1624, -1, True),
             (8192, 256, 768, -1, False), (256, 64, 24, 2, True)]
    for T, din, dout, act, need_dx in cases:
        x = torch.randn(T, din, device=DEV, generator=_g(41)).bfloat16()
        w = (0.05 * torch.randn(dout, din, device=DEV, generator=_g(42))).bfloat16()
        dy = torch.randn(T, dout, device=DEV, generator=_g(43)).bfloat16()
        pre = torch.randn(T, din, device=DEV, generator=_g(44)).bfloat16() if act >= 0 else None
        extra = torch.randn(4, dout, device=DEV, generator=_g(45))
        alpha = torch.tensor([0.5], device=DEV)
        want = esgpt.linear_bwd(dy, x, w, alpha, act, pre, need_dx, True, t0, extra)
        got = esgpt.linear_bwd(dy.clone(), x.clone(), w, alpha, act, pre, need_dx, True, t0, extra, t1)
        junk = [torch.full((T, max(din, dout)), 7.0, device=DEV, dtype=torch.bfloat16) for _ in range(3)]
        esgpt.weight_grad_join(t1)
        del junk
        for a, b, name in zip(want, got, ("dx", "dw", "db")):
            assert torch.equal(a, b), (T, din, dout, act, name)


@pytest.mark.parametrize("G", [1, 4])
def test_na_glue_ops_match_torch(env, G):
    """esgpt::na_split / na_assemble (+ backwards through StructuredAttention's autograd Functions) against the
    reference's torch formulation (structured_attention.py:63-156: where on the whole-event element, history = the
    masked ctx shifted by one event, cat), values and gradients bit for bit (pure data movement)."""
    from eventstreamgpt_amd.transformer.structured_attention import _NAAssemble, _NASplit

    B, L, D = 3, 37, 64
    x = torch.randn(B, L, G, D, device=DEV, generator=_g(20)).requires_grad_()
    em = torch.rand(B, L, device=DEV, generator=_g(21)) > 0.2
    w_ctx = torch.randn(D, D, device=DEV, generator=_g(22))
    d_out = torch.randn(B * L, G + 1, D, device=DEV, generator=_g(23))

    def ours():
        holder = {}
        per = _NASplit.apply(x, em, holder)
        ctx = torch.where(em[..., None], per @ w_ctx, 0.0)  # a stand-in sequence module (masked output)
        seq = _NAAssemble.apply(ctx, x, holder)
        return per, seq

    def ref():
        per = torch.where(em[..., None], x[:, :, -1, :], 0.0)
        ctx = torch.where(em[..., None], per @ w_ctx, 0.0)
        hist = torch.nn.functional.pad(ctx[:, :-1, :], (0, 0, 1, 0))
        seq = torch.cat((hist.unsqueeze(2), x[:, :, :-1, :], ctx.unsqueeze(2)), dim=2).reshape(B * L, G + 1, D)
        return per, seq

    p1, s1 = ours()
    (s1 * d_out).sum().backward()
    g1 = x.grad.clone()
    x.grad = None
    p2, s2 = ref()
    (s2 * d_out).sum().backward()
    assert torch.equal(p1, p2) and torch.equal(s1, s2)
    torch.testing.assert_close(g1, x.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("skip_T,mask_div,ydt", [(0, 1, torch.bfloat16), (5, 4, torch.bfloat16), (0, 1, torch.float32)])
def test_residual_op_matches_torch(env, skip_T, mask_div, ydt):
    """esgpt::residual: h = mask ? x[xr] + dropout(y) : 0 (InnerBlock's last residual with the NA event-mask where):
    exact without dropout; with dropout the kept / dropped elements scale y by 1/(1-p) or 0 and the backward applies
    the same mask to dh; x's gradient covers every row of x (zeros for the rows skip_T leaves out)."""
    esgpt, _ = env
    D = 128
    Bs, T = 6, 5
    N = Bs * (T - 1) if skip_T else Bs * T
    xrows = Bs * T
    x = torch.randn(xrows, D, device=DEV, generator=_g(30)).requires_grad_()
    y = torch.randn(N, D, device=DEV, generator=_g(31)).to(ydt).requires_grad_()
    mask = torch.rand(N // mask_div, device=DEV, generator=_g(32)) > 0.3
    rows = torch.arange(N, device=DEV)
    xr = (rows // (T - 1)) * T + 1 + rows % (T - 1) if skip_T else rows
    keep = mask.repeat_interleave(mask_div)[:, None]
    h = esgpt.residual(x, y, mask, mask_div, skip_T, 0.0, None)
    want = torch.where(keep, x[xr] + y.float(), 0.0)
    assert torch.equal(h, want)
    dh = torch.randn_like(h)
    h.backward(dh)
    gx = torch.zeros_like(x)
    gx[xr] = torch.where(keep, dh, 0.0)
    assert torch.equal(x.grad, gx)
    assert torch.equal(y.grad, torch.where(keep, dh, 0.0).to(ydt))
    # dropout: consistent masks forward / backward
    seed = torch.tensor([4242], dtype=torch.int64, device=DEV)
    x.grad = y.grad = None
    h = esgpt.residual(x, y, None, 1, skip_T, 0.25, seed)
    z = (h - x[xr]).detach() / y.float().detach()
    ok = (z - 0.0).abs() < 1e-3
    ok |= (z - 1 / 0.75).abs() < 1e-3
    assert bool(ok[y.float().abs() > 1e-3].all())
    h.backward(dh)
    kept = (z > 0.5) & (y.float().abs() > 1e-3)
    dyf = y.grad.float()
    assert torch.allclose(dyf[kept], (dh / 0.75).to(ydt).float()[kept], rtol=1e-2, atol=1e-3)
    assert bool((dyf[~kept & (y.float().abs() > 1e-3)] == 0).all())


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_residual_ln_skip_rows_equal_sliced_input(env, p):
    """esgpt::residual_ln with skip_T = T (the static_kv_first residual: x [Bs, T, D], output rows = every row but
    each sequence's first) equals the plain op on x[:, 1:] bit for bit, forward and backward (dx of the skipped rows
    zero)."""
    esgpt, _ = env
    Bs, T, D = 7, 5, 256
    x = torch.randn(Bs * T, D, device=DEV, generator=_g(40)).requires_grad_()
    y = torch.randn(Bs * (T - 1), D, device=DEV, generator=_g(41)).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(D, device=DEV, generator=_g(42))).requires_grad_()
    b = (0.1 * torch.randn(D, device=DEV, generator=_g(43))).requires_grad_()
    seed = torch.tensor([777], dtype=torch.int64, device=DEV) if p > 0 else None
    dout = torch.randn(Bs * (T - 1), D, device=DEV, generator=_g(44)).bfloat16()
    dh = torch.randn(Bs * (T - 1), D, device=DEV, generator=_g(45))
    h1, o1, _, _ = esgpt.residual_ln(x, y, None, w, b, None, p, seed, 1e-5, torch.bfloat16, T)
    torch.autograd.backward([h1, o1], [dh, dout])
    g1 = [t.grad.clone() for t in (x, y, w, b)]
    for t in (x, y, w, b):
        t.grad = None
    xs = x.view(Bs, T, D)[:, 1:].reshape(-1, D)
    h2, o2, _, _ = esgpt.residual_ln(xs, y, None, w, b, None, p, seed, 1e-5, torch.bfloat16)
    torch.autograd.backward([h2, o2], [dh, dout])
    assert torch.equal(h1, h2) and torch.equal(o1, o2)
    for a, c in zip(g1, (x.grad, y.grad, w.grad, b.grad)):
        assert torch.equal(a, c)
    assert bool((g1[0].view(Bs, T, D)[:, 0] == 0).all())
