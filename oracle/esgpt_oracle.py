"""ORACLE — test infrastructure only. Never imported by the product path.

A plain-PyTorch, fp32, CPU restatement of the reference's event-stream training step (Jwoo5/EventStreamGPT @
2025-01-14), written functionally over a ``state_dict``-keyed parameter dict so that it can be fed the exact
weights of a product model (or of a reference model) and differentiated with autograd.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, and
only as the checker / CPU baseline.

Pinning: the restatement is checked against golden vectors produced by running the reference itself in the
survey container (``tests/golden/make_golden.py``; fixtures in ``tests/golden/*.pt``) and against the reference
tests' known answers (``tests/golden/known_answers.json``). The LogNormalMixture TTE lives in the third-party
``pytorch-lognormal-mixture==0.0.1`` (reference ``env.yml:409``; absent here): its published algorithm is
restated in ``lnm_log_prob``; the (mean_log, std_log) = (0, 1) branch is pinned by the reference's known answer
LL = -7.6554941334115565, the affine branch is pinned only against the stub restatement that ran the reference
(parity unpinned against upstream code for that branch).

``cfg`` is any object with the reference ``StructuredTransformerConfig`` attribute names. ``batch`` is any object
supporting ``batch["field"]`` for the ``PytorchBatch`` fields.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

FMIN = torch.finfo(torch.float32).min
TINY = torch.finfo(torch.float32).tiny


def _lin(p, name, x):
    w = p[name + ".weight"]
    b = p.get(name + ".bias")
    return F.linear(x, w, b)


def _ln(p, name, x, eps):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


# --------------------------------------------------------------------------------------------------------------
# Embedding: EventStream/data/data_embedding_layer.py
# --------------------------------------------------------------------------------------------------------------
def meas_index_normalization(meas: torch.Tensor) -> torch.Tensor:
    """``get_measurement_index_normalziation`` (``data_embedding_layer.py:314-349``): each distinct non-zero
    measurement index in a row gets total weight 1/(#distinct), split evenly over its occurrences."""
    eq = meas.unsqueeze(-1) == meas.unsqueeze(-2)  # [..., M, M]
    cnt = eq.sum(-1).to(torch.float32)
    w = torch.where(meas == 0, torch.zeros_like(cnt), 1.0 / cnt)
    s = w.sum(-1, keepdim=True)
    s = torch.where(s == 0, torch.ones_like(s), s)
    return w / s


def embedding_bag_sum(table, idx, w):
    """``nn.EmbeddingBag(mode="sum", padding_idx=0)`` with per-sample weights: index 0 contributes nothing."""
    rows = table[idx]  # [..., M, D]
    w = torch.where(idx == 0, torch.zeros_like(w), w)
    return (rows * w.unsqueeze(-1)).sum(-2)


def _weights(ew):
    ew = dict(ew)
    s, d = ew["static_weight"], ew["dynamic_weight"]
    c, n = ew["categorical_weight"], ew["numerical_weight"]
    return s / (s + d), d / (s + d), c / (c + n), n / (c + n)


def embed_bags(p, prefix, cfg_emb, idx, meas, values=None, values_mask=None, cat_mask=None):
    """``_embed`` → ``_joint_embed`` (``:351-388``) or ``_split_embed`` (``:390-450``) on [..., M] bags."""
    sw, dw, cw, nw = _weights(cfg_emb)
    norm = meas_index_normalization(meas) if cfg_emb["do_normalize_by_measurement_index"] else None
    if cfg_emb["mode"] == "joint":
        if values is None:
            v = torch.ones_like(idx, dtype=torch.float32)
        else:
            v = torch.where(values_mask, values, torch.ones_like(values))
        if norm is not None:
            v = v * norm
        return embedding_bag_sum(p[prefix + "embed_layer.weight"], idx, v)
    cv = torch.ones_like(idx, dtype=torch.float32)
    if cat_mask is not None:
        cv = torch.where(cat_mask, cv, torch.zeros_like(cv))
    if norm is not None:
        cv = cv * norm
    cat = _lin(p, prefix + "cat_proj", embedding_bag_sum(p[prefix + "categorical_embed_layer.weight"], idx, cv))
    if values is None:
        return cat  # static path: no categorical_weight (data_embedding_layer.py:441-442)
    nv = torch.where(values_mask, values, torch.zeros_like(values))
    if norm is not None:
        nv = nv * norm
    num = _lin(p, prefix + "num_proj", embedding_bag_sum(p[prefix + "numerical_embed_layer.weight"], idx, nv))
    return cw * cat + nw * num


def bucket_masks(meas, groups):
    """``_split_batch_into_measurement_index_buckets`` (``:505-561``) → bool [B,L,G,M] (cat, num)."""
    cats, nums = [], []
    for gi, group in enumerate(groups):
        if len(group) == 0 and gi > 0:
            raise ValueError(f"Empty measurement index group: {group} at index {gi}!")
        cm = torch.zeros_like(meas, dtype=torch.bool)
        nm = torch.zeros_like(meas, dtype=torch.bool)
        for entry in group:
            if isinstance(entry, (tuple, list)):
                mi, mode = entry
            else:
                mi, mode = entry, "categorical_and_numerical"
            hit = meas == mi
            if mode in ("categorical_and_numerical", "categorical_only"):
                cm = cm | hit
            if mode in ("categorical_and_numerical", "numerical_only"):
                nm = nm | hit
        cats.append(cm)
        nums.append(nm)
    return torch.stack(cats, -2), torch.stack(nums, -2)


def data_embedding(p, prefix, cfg_emb, batch, groups=None):
    """``DataEmbeddingLayer.forward`` (``:609-708``) → [B,L,D] or [B,L,G,D]."""
    idx, meas = batch["dynamic_indices"], batch["dynamic_measurement_indices"]
    vals, vmask = batch["dynamic_values"], batch["dynamic_values_mask"]
    B, L, M = idx.shape
    if groups:
        cm, nm = bucket_masks(meas, groups)
        G = cm.shape[-2]
        ex = lambda t: t.unsqueeze(-2).expand(B, L, G, M)  # noqa: E731
        emb = embed_bags(p, prefix, cfg_emb, ex(idx), ex(meas), ex(vals), ex(vmask) & nm, cm)
    else:
        emb = embed_bags(p, prefix, cfg_emb, idx, meas, vals, vmask, None)
    mask = batch["event_mask"]
    while mask.dim() < emb.dim():
        mask = mask.unsqueeze(-1)
    emb = torch.where(mask, emb, torch.zeros_like(emb))
    if cfg_emb["static_embedding_mode"] == "drop":
        return emb
    sw, dw, _, _ = _weights(cfg_emb)
    st = embed_bags(p, prefix, cfg_emb, batch["static_indices"], batch["static_measurement_indices"]).unsqueeze(1)
    if groups:
        st = st.unsqueeze(2)
    emb = dw * emb + sw * st
    return torch.where(mask, emb, torch.zeros_like(emb))


def time_from_deltas(event_mask, time_delta):
    """``transformer.py:539-561``: exclusive cumsum of masked deltas (CPU cumsum accumulates in double)."""
    td = torch.where(event_mask, time_delta, torch.zeros_like(time_delta))
    return torch.cat([torch.zeros_like(td[:, :1]), td.cumsum(-1)[:, :-1]], dim=1)


def temporal_encoding(p, prefix, batch, D):
    """``TemporalPositionEncoding.forward`` (``:594-619``)."""
    t = batch.get("time", None) if hasattr(batch, "get") else None
    if t is None:
        t = time_from_deltas(batch["event_mask"], batch["time_delta"])
    t = t.unsqueeze(-1)
    out = torch.zeros(t.shape[0], t.shape[1], D)
    out[:, :, 0::2] = torch.sin(t * p[prefix + "sin_div_term"])
    out[:, :, 1::2] = torch.cos(t * p[prefix + "cos_div_term"])
    return out


def div_terms(D: int, max_timepoint: float = 10000.0):
    """The frozen ``sin_div_term`` / ``cos_div_term`` parameters (``transformer.py:578-592``)."""
    div = torch.exp(torch.arange(0, D, 2) * (-math.log(max_timepoint) / D))
    return div, (div if D % 2 == 0 else div[:-1])


def emb_cfg(cfg) -> dict:
    return dict(
        mode="split" if cfg.categorical_embedding_dim is not None else "joint",
        do_normalize_by_measurement_index=bool(cfg.do_normalize_by_measurement_index),
        static_embedding_mode=str(cfg.static_embedding_mode),
        static_weight=cfg.static_embedding_weight, dynamic_weight=cfg.dynamic_embedding_weight,
        categorical_weight=cfg.categorical_embedding_weight, numerical_weight=cfg.numerical_embedding_weight,
    )


def dep_graph_groups(cfg):
    """Measurement-name groups → measurement-index groups (``transformer.py:866-884``)."""
    out = []
    for level in cfg.measurements_per_dep_graph_level:
        grp = []
        for m in level:
            if isinstance(m, str):
                grp.append(cfg.measurements_idxmap[m])
            else:
                grp.append((cfg.measurements_idxmap[m[0]], str(m[1])))
        out.append(grp)
    return out


# --------------------------------------------------------------------------------------------------------------
# Transformer: EventStream/transformer/transformer.py
# --------------------------------------------------------------------------------------------------------------
def causal_band(Lk: int, attention_type: str, window: int | None) -> torch.Tensor:
    """The uint8 ``bias`` buffer as bool (``:109-119``): key j allowed for query i iff j <= i (and i-j < w)."""
    tril = torch.tril(torch.ones(Lk, Lk, dtype=torch.bool))
    if attention_type == "local":
        tril = tril & ~torch.tril(tril, -window)
    return tril


def self_attention(p, pre, x, cfg, attn_type, window, key_mask=None, static_kv_first=False):
    """``InnerSelfAttention.forward`` + ``_attn`` (``:171-282``), no dropout, no cache."""
    B, T, D = x.shape
    H, hd = cfg.num_attention_heads, cfg.head_dim
    q = _lin(p, pre + "q_proj", x).view(B, T, H, hd).permute(0, 2, 1, 3)
    k = _lin(p, pre + "k_proj", x).view(B, T, H, hd).permute(0, 2, 1, 3)
    v = _lin(p, pre + "v_proj", x).view(B, T, H, hd).permute(0, 2, 1, 3)
    if static_kv_first:
        q = q[:, :, 1:, :]
    Lq, Lk = q.shape[-2], k.shape[-2]
    s = torch.matmul(q, k.transpose(-1, -2))  # NB: no 1/sqrt(hd) scaling in the reference
    band = causal_band(Lk, attn_type, window)[Lk - Lq: Lk, :Lk]
    s = torch.where(band, s, torch.tensor(FMIN))
    if key_mask is not None:
        s = s + (1.0 - key_mask[:, None, None, :].float()) * FMIN
    a = torch.softmax(s, dim=-1)
    o = torch.matmul(a, v).permute(0, 2, 1, 3).reshape(B, Lq, D)
    return _lin(p, pre + "out_proj", o)


def inner_attention(p, pre, x, cfg, layer, is_seq, key_mask=None, static_kv_first=False):
    """``InnerAttention.forward`` (``:325-358``): LN then attention; no residual."""
    types = cfg.seq_attention_layers if is_seq else cfg.dep_graph_attention_layers
    at = types[layer]
    w = (cfg.seq_window_size if is_seq else cfg.dep_graph_window_size) if at == "local" else None
    h = _ln(p, pre + "layer_norm", x, cfg.layer_norm_epsilon)
    return self_attention(p, pre + "attention.", h, cfg, at, w, key_mask, static_kv_first)


def inner_mlp(p, pre, x, cfg):
    """``InnerMLP`` (``:361-391``): c_fc → act (erf GELU for "gelu") → c_proj."""
    h = _lin(p, pre + "c_fc", x)
    act = cfg.activation_function
    if act == "gelu":
        h = F.gelu(h)
    elif act in ("gelu_new", "gelu_pytorch_tanh"):
        h = F.gelu(h, approximate="tanh")
    elif act == "relu":
        h = F.relu(h)
    else:
        raise ValueError(f"oracle: unsupported activation {act}")
    return _lin(p, pre + "c_proj", h)


def inner_block(p, pre, x, cfg, layer, is_seq, key_mask=None, static_kv_first=False):
    """``InnerBlock.forward`` (``:409-461``)."""
    resid = x[:, 1:, :] if static_kv_first else x
    a = inner_attention(p, pre + "attn.", x, cfg, layer, is_seq, key_mask, static_kv_first)
    h = a + resid
    return h + inner_mlp(p, pre + "mlp.", _ln(p, pre + "layer_norm", h, cfg.layer_norm_epsilon), cfg)


def ci_encoder(p, cfg, batch, pre="encoder."):
    """``ConditionallyIndependentPointProcessTransformer.forward`` (``:708-848``), training path."""
    D = cfg.hidden_size
    em = batch["event_mask"]
    x = data_embedding(p, pre + "input_layer.data_embedding_layer.", emb_cfg(cfg), batch)
    x = x + temporal_encoding(p, pre + "input_layer.time_embedding_layer.", batch, D)
    x = torch.where(em.unsqueeze(-1), x, torch.zeros_like(x))
    for i in range(cfg.num_hidden_layers):
        x = inner_block(p, f"{pre}h.{i}.", x, cfg, i, True, key_mask=em)
        x = torch.where(em.unsqueeze(-1), x, torch.zeros_like(x))
    return _ln(p, pre + "ln_f", x, cfg.layer_norm_epsilon)


def na_encoder(p, cfg, batch, pre="encoder."):
    """``NestedAttentionPointProcessTransformer.forward`` (``:975-1233``) + ``StructuredAttention.forward``
    (``structured_attention.py:28-219``), training path (no cache)."""
    D = cfg.hidden_size
    em = batch["event_mask"]
    x = data_embedding(p, pre + "input_layer.data_embedding_layer.", emb_cfg(cfg), batch, dep_graph_groups(cfg))
    t = temporal_encoding(p, pre + "input_layer.time_embedding_layer.", batch, D)
    x = torch.cat([x[:, :, :1] + t.unsqueeze(2), x[:, :, 1:]], dim=2).cumsum(dim=2)
    x = torch.where(em[..., None, None], x, torch.zeros_like(x))
    B, L, G, _ = x.shape
    flat = em.reshape(-1)
    for i in range(cfg.num_hidden_layers):
        bp = f"{pre}h.{i}.block."
        per_event = torch.where(em.unsqueeze(-1), x[:, :, -1, :], torch.zeros_like(x[:, :, -1, :]))
        if cfg.do_full_block_in_seq_attention:
            ctx = inner_block(p, bp + "seq_module.", per_event, cfg, i, True, key_mask=em)
        else:
            ctx = inner_attention(p, bp + "seq_module.", per_event, cfg, i, True, key_mask=em)
        ctx = torch.where(em.unsqueeze(-1), ctx, torch.zeros_like(ctx))
        hist = torch.cat([torch.zeros_like(ctx[:, :1]), ctx[:, :-1]], dim=1)
        dg = torch.cat([hist.unsqueeze(2), x[:, :, :-1], ctx.unsqueeze(2)], dim=2)  # last el := ctx
        dg = dg.reshape(B * L, G + 1, D)[flat]
        if cfg.do_full_block_in_dep_graph_attention:
            out = inner_block(p, bp + "dep_graph_module.", dg, cfg, i, False, None, static_kv_first=True)
        else:
            out = inner_attention(p, bp + "dep_graph_module.", dg, cfg, i, False, None, static_kv_first=True)
        full = torch.zeros(B * L, G, D, dtype=out.dtype)
        full = full.index_put((flat.nonzero().squeeze(-1),), out)
        x = full.reshape(B, L, G, D)
    return _ln(p, pre + "ln_f", x, cfg.layer_norm_epsilon)


# --------------------------------------------------------------------------------------------------------------
# Losses: EventStream/transformer/{model_output.py,generative_layers.py,utils.py}
# --------------------------------------------------------------------------------------------------------------
def safe_weighted_avg(X, w):
    """``utils.py:134-206``."""
    if w.dim() < X.dim():
        w = w.unsqueeze(-2).expand_as(X)
    w = w.float()
    den = w.sum(-1)
    safe = torch.where(den > 0, den, torch.ones_like(den))
    return torch.where(den > 0, (X * w).sum(-1) / safe, torch.zeros_like(den)), den


def weighted_loss(loss_per_event, mask):
    """``utils.py:209-234``: mean over subjects with events of per-subject mean."""
    per_subj, n = safe_weighted_avg(loss_per_event, mask)
    return safe_weighted_avg(per_subj, n > 0)[0]


def lnm_log_prob(params, x, mean_log, std_log):
    """LogNormalMixture log-density (third-party ``pytorch_lognormal_mixture``; see module docstring).

    params [..., 3K] from ``LogNormalMixtureTTELayer.proj``: locs = p[0::3], log_scales = p[1::3],
    log_weights = p[2::3] (``generative_layers.py:53-59``). y = (ln x − μ)/σ when (μ,σ) ≠ (0,1).
    """
    locs, log_scales, log_w = params[..., 0::3], params[..., 1::3], params[..., 2::3]
    lx = torch.log(x)
    affine = not (mean_log == 0.0 and std_log == 1.0)
    y = (lx - mean_log) / std_log if affine else lx
    comp = torch.distributions.Normal(locs, log_scales.exp()).log_prob(y.unsqueeze(-1))
    lp = torch.logsumexp(torch.log_softmax(log_w, dim=-1) + comp, dim=-1)
    lp = lp - lx  # Exp transform Jacobian
    if affine:
        lp = lp - math.log(abs(std_log))
    return lp


def tte_log_likelihood(p, pre, cfg, batch, enc):
    """``get_TTE_outputs`` (``model_output.py:1311-1372``) → scalar mean-over-subjects LL."""
    em = batch["event_mask"]
    obs = em[:, 1:] & em[:, :-1]
    td = batch["time_delta"][:, :-1]
    true = torch.where(obs, td, torch.ones_like(td))
    true = torch.cat([true, torch.ones_like(true[:, -1:])], dim=-1)
    obs = torch.cat([obs, torch.zeros_like(obs[:, -1:])], dim=-1)
    z = _lin(p, pre + "TTE_layer.proj", enc)
    if cfg.TTE_generation_layer_type == "exponential":
        rate = (F.elu(z) + 1 + TINY).squeeze(-1)
        ll = torch.log(rate) - rate * true
    else:
        ll = lnm_log_prob(z, true, cfg.mean_log_inter_event_time_min, cfg.std_log_inter_event_time_min)
    if torch.isnan(ll).any():
        raise ValueError("NaNs in TTE_LL")
    cnt = obs.float().sum(-1)
    if (cnt == 0).any():
        raise ValueError("No observed time-to-event for >= 1 patient in batch")
    return ((ll * obs.float()).sum(-1) / cnt).mean()


def _vocab_end(cfg, start):
    return min(o for o in list(cfg.vocab_offsets_by_measurement.values()) + [cfg.vocab_size] if o > start)


def classification_losses(p, pre, cfg, batch, enc, valid):
    """``get_classification_outputs`` (``model_output.py:1374-1549``) → {measurement: loss}."""
    out = {}
    if not valid:
        return out
    is_obs = _lin(p, pre + "IsObservedLayer", enc)
    scores_all = _lin(p, pre + "ClassificationLayer", enc)
    idx, meas = batch["dynamic_indices"], batch["dynamic_measurement_indices"]
    for mode in ("single_label_classification", "multi_label_classification"):
        for m in cfg.measurements_per_generative_mode.get(mode, []):
            if m not in valid:
                continue
            mi = cfg.measurements_idxmap[m]
            vs = cfg.vocab_offsets_by_measurement[m]
            ve = _vocab_end(cfg, vs)
            scores = scores_all[:, :, vs:ve]
            hit = meas == mi
            em = batch["event_mask"]
            if mode == "single_label_classification":
                has = hit.any(-1)
                obs_loss = F.binary_cross_entropy_with_logits(is_obs[:, :, mi - 1], has.float(), reduction="none")
                labels = ((idx * hit.long()).sum(-1) - vs) * has.long()
                lpe = F.cross_entropy(scores.transpose(1, 2), labels, reduction="none") + obs_loss
                out[m] = weighted_loss(lpe, em & has)
            else:
                lab = torch.where(hit, idx - vs + 1, torch.zeros_like(idx))
                y = torch.zeros(scores.shape[0], scores.shape[1], 1 + scores.shape[2]).scatter(2, lab, 1.0)[..., 1:]
                lpe = F.binary_cross_entropy_with_logits(scores, y, reduction="none").mean(-1)
                out[m] = weighted_loss(lpe, em)
    return out


def _normal_nll(mean, std, x):
    return -torch.distributions.Normal(mean, std).log_prob(x)


def regression_losses(p, pre, cfg, batch, enc, valid):
    """``get_regression_outputs`` (``model_output.py:1551-1721``) → {measurement: loss}."""
    out = {}
    if not valid:
        return out
    is_obs = _lin(p, pre + "IsObservedLayer", enc)
    idx, meas = batch["dynamic_indices"], batch["dynamic_measurement_indices"]
    vals, vmask, em = batch["dynamic_values"], batch["dynamic_values_mask"], batch["event_mask"]
    for m in cfg.measurements_per_generative_mode.get("multivariate_regression", []):
        if m not in valid:
            continue
        mi = cfg.measurements_idxmap[m]
        vs = cfg.vocab_offsets_by_measurement[m]
        sel = (meas == mi) & vmask
        gidx = torch.where(sel, idx - vs, torch.zeros_like(idx))
        z = _lin(p, pre + f"regression_layers.{m}.proj", enc)
        mean = z[..., 0::2].gather(-1, gidx)
        std = (F.elu(z[..., 1::2]) + 1 + TINY).gather(-1, gidx)
        x = torch.where(sel, vals, torch.zeros_like(vals))
        lpe, _ = safe_weighted_avg(_normal_nll(mean, std, x), sel)
        out[m] = weighted_loss(lpe, em & sel.any(-1))
    for m in cfg.measurements_per_generative_mode.get("univariate_regression", []):
        if m not in valid:
            continue
        mi = cfg.measurements_idxmap[m]
        hit = meas == mi
        obs_loss = F.binary_cross_entropy_with_logits(is_obs[:, :, mi - 1], hit.any(-1).float(), reduction="none")
        lab = hit & vmask
        has = lab.any(-1)
        z = _lin(p, pre + f"regression_layers.{m}.proj", enc)
        mean, std = z[..., 0:1], F.elu(z[..., 1:2]) + 1 + TINY
        x = (torch.where(lab, vals, torch.zeros_like(vals)).sum(-1) * has.float()).unsqueeze(-1)
        lpe = _normal_nll(mean, std, x).squeeze(-1)
        out[m] = weighted_loss(lpe + obs_loss, em & has)
    return out


def _regression_measurements(cfg):
    return set(cfg.measurements_per_generative_mode.get("multivariate_regression", [])
               + cfg.measurements_per_generative_mode.get("univariate_regression", []))


def _classification_measurements(cfg):
    return set(cfg.measurements_per_generative_mode.get("single_label_classification", [])
               + cfg.measurements_per_generative_mode.get("multi_label_classification", []))


def ci_output_losses(p, cfg, batch, enc, pre="output_layer."):
    """``ConditionallyIndependentGenerativeOutputLayer.forward`` (``conditionally_independent_model.py:45-161``)."""
    shifted = torch.cat([torch.zeros_like(enc[:, :1]), enc[:, :-1]], dim=1)
    cls = classification_losses(p, pre, cfg, batch, shifted, _classification_measurements(cfg))
    reg = regression_losses(p, pre, cfg, batch, shifted, _regression_measurements(cfg))
    tte = tte_log_likelihood(p, pre, cfg, batch, enc)
    return cls, reg, tte


def na_output_losses(p, cfg, batch, enc, pre="output_layer."):
    """``NestedAttentionGenerativeOutputLayer.forward`` (``nested_attention_model.py:47-228``)."""
    cls_all, reg_all = _classification_measurements(cfg), _regression_measurements(cfg)
    cls, reg = {}, {}
    G = enc.shape[2]
    for i in range(1, G):
        cat_in, num_in = set(), set()
        for m in cfg.measurements_per_dep_graph_level[i]:
            if isinstance(m, (tuple, list)):
                name, mode = m[0], str(m[1])
            else:
                name, mode = m, "categorical_and_numerical"
            if mode in ("categorical_and_numerical", "categorical_only"):
                cat_in.add(name)
            if mode in ("categorical_and_numerical", "numerical_only"):
                num_in.add(name)
        lvl = enc[:, :, i - 1, :]
        cls.update(classification_losses(p, pre, cfg, batch, lvl, cat_in & cls_all))
        reg.update(regression_losses(p, pre, cfg, batch, lvl, num_in & reg_all))
    tte = tte_log_likelihood(p, pre, cfg, batch, enc[:, :, -1, :])
    return cls, reg, tte


def model_losses(p, cfg, batch, pre="") -> dict:
    """Full ``CIPPT``/``NAPPT`` forward → {"loss", "classification", "regression", "tte_ll", "encoded"}.

    loss = Σ classification + Σ regression − TTE LL (``conditionally_independent_model.py:132-136``). Dict
    iteration follows the reference: classification in ``classification_mode_per_measurement`` order.
    """
    if str(cfg.structured_event_processing_mode) == "conditionally_independent":
        enc = ci_encoder(p, cfg, batch, pre + "encoder.")
        cls, reg, tte = ci_output_losses(p, cfg, batch, enc, pre + "output_layer.")
    else:
        enc = na_encoder(p, cfg, batch, pre + "encoder.")
        cls, reg, tte = na_output_losses(p, cfg, batch, enc, pre + "output_layer.")
    loss = sum(cls.values()) + sum(reg.values()) - tte
    return {"loss": loss, "classification": cls, "regression": reg, "tte_ll": tte, "encoded": enc}


def stream_classification_loss(p, cfg, batch, labels, pooling: str, binary: bool, pre: str = ""):
    """``ESTForStreamClassification.forward`` (``fine_tuning_model.py:54-91``): encoder (last dep-graph level for
    NA), pooling over the sequence (``cls`` / ``last`` / masked ``max`` / masked ``mean``, ``utils.py:61-207``),
    ``logit_layer`` and BCE-with-logits (binary) or cross-entropy. Returns (loss, logits)."""
    if str(cfg.structured_event_processing_mode) == "conditionally_independent":
        enc = ci_encoder(p, cfg, batch, pre + "encoder.")
    else:
        enc = na_encoder(p, cfg, batch, pre + "encoder.")[:, :, -1, :]
    x = enc.transpose(1, 2)  # [B, D, L], the reference's layout for the masked reductions
    em = batch["event_mask"]
    if pooling == "cls":
        pooled = x[:, :, 0]
    elif pooling == "last":
        pooled = x[:, :, -1]
    elif pooling == "max":
        m = torch.where(em.unsqueeze(-2).expand_as(x), x, torch.full_like(x, -float("inf"))).max(-1)[0]
        pooled = torch.nan_to_num(m, nan=None, posinf=None, neginf=0.0)
    elif pooling == "mean":
        pooled = safe_weighted_avg(x, em.unsqueeze(-2).expand_as(x).float())[0]
    else:
        raise ValueError(pooling)
    logits = _lin(p, pre + "logit_layer", pooled).squeeze(-1)
    if binary:
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, labels)
    else:
        loss = torch.nn.functional.cross_entropy(logits, labels)
    return loss, logits


# --------------------------------------------------------------------------------------------------------------
# Optimiser: generative_modeling.py:460-485 (AdamW + transformers.get_polynomial_decay_schedule_with_warmup)
# --------------------------------------------------------------------------------------------------------------
def poly_decay_lr(step: int, init_lr: float, end_lr: float, warmup: int, total: int, power: float) -> float:
    """LR multiplier schedule of ``get_polynomial_decay_schedule_with_warmup`` (transformers), × init_lr."""
    if step < warmup:
        return init_lr * float(step) / float(max(1, warmup))
    if step > total:
        return end_lr
    rng = init_lr - end_lr
    rem = 1 - (step - warmup) / (total - warmup)
    return rng * rem**power + end_lr


def adamw_step(params: dict, grads: dict, state: dict, lr: float, wd: float,
               betas=(0.9, 0.999), eps: float = 1e-8):
    """One ``torch.optim.AdamW`` step (decoupled weight decay), in place on ``params``."""
    b1, b2 = betas
    state["t"] = state.get("t", 0) + 1
    t = state["t"]
    for k, w in params.items():
        g = grads.get(k)
        if g is None:
            continue
        m = state.setdefault("m_" + k, torch.zeros_like(w))
        v = state.setdefault("v_" + k, torch.zeros_like(w))
        w.mul_(1 - lr * wd)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1**t
        bc2 = 1 - b2**t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        w.addcdiv_(m, denom, value=-lr / bc1)
