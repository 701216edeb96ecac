"""``StructuredAttention`` — drop-in for ``EventStream/transformer/structured_attention.py:7-219``.

Differences in mechanics (same results): padded events are NOT compacted out with boolean indexing (a device→host
sync and data-dependent shapes in the reference, ``:87-96,158-165,186-193``); every (subject, event) runs through
the dependency-graph module — its sequences are independent — and the outputs of padded events are zeroed, which
is exactly what the reference's scatter into a zero tensor produces. This keeps the step shape-static (capturable
into a HIP graph).

Generation with caches (``prepend_graph_with_history_embeddings`` / ``update_last_graph_el_to_history_embedding``
False, set by the encoder from ``dep_graph_el_generation_target``): the three cases of ``:63-156`` — prefill
(history prepended, the last graph element replaced by the contextualised event), a new event's whole-event
element (no history: it is in the dependency-graph cache; its contextualised version replaces it) and a new graph
element (no sequence module at all).
"""
from __future__ import annotations

from typing import Any

import torch


class _SplitLast(torch.autograd.Function):
    """x [..., G, D] -> (x[..., :G-1, :], x[..., G-1, :]) as contiguous tensors whose backward is ONE cat of the two
    incoming gradients (autograd's slice / select backwards would zero-fill a full-size gradient for each and add
    them). A missing incoming gradient counts as zeros."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x[..., :-1, :].contiguous(), x[..., -1, :].contiguous()

    @staticmethod
    def backward(ctx, d_head, d_last):
        shape = ctx.shape
        ref = d_head if d_head is not None else d_last
        if d_head is None:
            d_head = ref.new_zeros(shape[:-2] + (shape[-2] - 1, shape[-1]))
        if d_last is None:
            d_last = ref.new_zeros(shape[:-2] + (shape[-1],))
        return torch.cat((d_head, d_last.unsqueeze(-2)), dim=-2)


def split_last_level(x: torch.Tensor):
    """(all but the last dependency-graph level, the last level) of x [..., G, D], without zero-filled backwards."""
    return _SplitLast.apply(x)


class _Assemble(torch.autograd.Function):
    """The dependency-graph sequence [h_{i-1}, e_{i,1}, ..., e_{i,G-1}, ctx_i] per event (structured_attention.py:
    125-149): history = ctx shifted by one event (zeros first), head = the graph elements but the last, ctx = the
    contextualised event. Backward: d head = a view of the incoming gradient, d ctx = its last element plus the
    history slot of the next event — no zero-filled slice gradients."""

    @staticmethod
    def forward(ctx_, ctx, head):
        history = torch.nn.functional.pad(ctx[:, :-1, :], (0, 0, 1, 0))
        return torch.cat((history.unsqueeze(2), head, ctx.unsqueeze(2)), dim=2)

    @staticmethod
    def backward(ctx_, d):
        d_ctx = d[:, :, -1, :].clone()
        d_ctx[:, :-1, :] += d[:, 1:, 0, :]
        return d_ctx, d[:, :, 1:-1, :]


class _NASplit(torch.autograd.Function):
    """per_event = event_mask ? x[:, :, G-1] : 0 (``esgpt::na_split``). The gradient of x is assembled in ONE buffer:
    levels 0 .. G-2 come from ``_NAAssemble``'s backward (which always runs first: the sequence module's input
    gradient depends on it) through ``holder``; this backward writes level G-1 into it (``esgpt::na_split_bwd_``)."""

    @staticmethod
    def forward(ctx, x, event_mask, holder):
        from ..kernels import _ops

        ctx.save_for_backward(event_mask)
        ctx.holder, ctx.shape = holder, x.shape
        return _ops().na_split(x, event_mask)

    @staticmethod
    def backward(ctx, dper):
        from ..kernels import _ops

        (em,) = ctx.saved_tensors
        dx = ctx.holder.pop("dx", None)
        if dx is None:  # the dependency-graph sequence got no gradient: its levels contribute zeros
            dx = dper.new_zeros(ctx.shape, dtype=torch.float32)
        _ops().na_split_bwd_(dper, em, dx)
        return dx, None, None


class _NAAssemble(torch.autograd.Function):
    """The dependency-graph sequence [h_{i-1}, e_{i,1} .. e_{i,G-1}, ctx_i] per event (structured_attention.py:
    125-149) in one kernel (``esgpt::na_assemble``): ctx (the masked sequence-module output) shifted by one event
    for the history, x's first G-1 levels, ctx. Backward (``esgpt::na_assemble_bwd``): d ctx, and levels 0 .. G-2
    of d x handed to ``_NASplit`` through ``holder`` (x's gradient is returned there, not here)."""

    @staticmethod
    def forward(ctx, ctx_emb, x, holder):
        from ..kernels import _ops

        ctx.holder, ctx.BL = holder, (x.shape[0], x.shape[1])
        return _ops().na_assemble(ctx_emb, x)

    @staticmethod
    def backward(ctx, dseq):
        from ..kernels import _ops

        dctx, dx = _ops().na_assemble_bwd(dseq.contiguous(), ctx.BL[0], ctx.BL[1])
        ctx.holder["dx"] = dx
        return dctx, None, None


def _glue_fast_path(module, hidden_states, event_mask, seq_kwargs, dep_kwargs, prepend, update_last) -> bool:
    """The training path (history prepended, no caches) with both modules full InnerBlocks on a HIP f32 tensor:
    the split / assemble / mask steps run as the esgpt glue kernels (not when ``fused.ENABLED`` is off: that is the
    plain-PyTorch module path the fused-block tests compare against)."""
    from .. import fused
    from .transformer import InnerBlock

    return (fused.ENABLED and prepend and update_last and event_mask is not None and not seq_kwargs and not dep_kwargs
            and isinstance(module.seq_module, InnerBlock) and isinstance(module.dep_graph_module, InnerBlock)
            and hidden_states.is_cuda and hidden_states.dtype == torch.float32 and hidden_states.shape[-1] % 4 == 0)


class StructuredAttention(torch.nn.Module):
    def __init__(self, seq_module: torch.nn.Module, dep_graph_module: torch.nn.Module):
        super().__init__()
        self.seq_module = seq_module
        self.dep_graph_module = dep_graph_module

    def forward(self, hidden_states: torch.Tensor, seq_attention_mask: torch.Tensor | None = None,
                event_mask: torch.Tensor | None = None, seq_module_kwargs: dict[str, Any] | None = None,
                dep_graph_module_kwargs: dict[str, Any] | None = None,
                prepend_graph_with_history_embeddings: bool = True,
                update_last_graph_el_to_history_embedding: bool = True):
        seq_module_kwargs = dict(seq_module_kwargs or {})
        dep_graph_module_kwargs = dict(dep_graph_module_kwargs or {})
        bsz, seq_len, dep_graph_len, hidden_size = hidden_states.shape
        m3 = None if event_mask is None else event_mask.unsqueeze(-1)
        seq_ret = None

        if _glue_fast_path(self, hidden_states, event_mask, seq_module_kwargs, dep_graph_module_kwargs,
                           prepend_graph_with_history_embeddings, update_last_graph_el_to_history_embedding):
            kpm = (seq_attention_mask.reshape(bsz, -1) == 0) if seq_attention_mask is not None else event_mask
            em = event_mask.contiguous()
            x = hidden_states.contiguous()
            holder: dict = {}
            per_event = _NASplit.apply(x, em, holder)
            ctx, seq_ret = self.seq_module(per_event, key_padding_mask=kpm, out_row_mask=em.reshape(-1))
            dep_graph_seq = _NAAssemble.apply(ctx, x, holder)
            out, dep_ret = self.dep_graph_module(dep_graph_seq, attention_mask=None, static_kv_first=True,
                                                 out_row_mask=em.reshape(-1), out_mask_div=dep_graph_len)
            return (out.reshape(bsz, seq_len, dep_graph_len, hidden_size),
                    {"seq_module": seq_ret, "dep_graph_module": dep_ret})

        if prepend_graph_with_history_embeddings or update_last_graph_el_to_history_embedding:
            # key padding of the sequence module: the additive mask covers past + new events when a cache is used
            if seq_attention_mask is not None:
                kpm = seq_attention_mask.reshape(bsz, -1) == 0
            else:
                kpm = event_mask
            head, per_event = split_last_level(hidden_states)
            if m3 is not None:
                per_event = torch.where(m3, per_event, 0.0)
            ctx = self.seq_module(per_event, key_padding_mask=kpm, **seq_module_kwargs)
            if isinstance(ctx, tuple):
                ctx, seq_ret = ctx
            if m3 is not None:
                ctx = torch.where(m3, ctx, 0.0)
            if prepend_graph_with_history_embeddings:
                # [h_{i-1}, e_{i,1}, ..., e_{i,G-1}, ctx_i], h_{i-1} = ctx_{i-1} (zeros first): the last graph element
                # is replaced by the contextualised event (structured_attention.py:125-149).
                dep_graph_seq = _Assemble.apply(ctx, head)
                static_kv_first = True
            else:
                dep_graph_seq = torch.cat((head, ctx.unsqueeze(2)), dim=2)
                static_kv_first = False
        else:
            dep_graph_seq = hidden_states
            static_kv_first = False

        G1 = dep_graph_seq.shape[2]
        dep_graph_seq = dep_graph_seq.reshape(bsz * seq_len, G1, hidden_size)
        out = self.dep_graph_module(dep_graph_seq, attention_mask=None, static_kv_first=static_kv_first,
                                    **dep_graph_module_kwargs)
        dep_ret = None
        if isinstance(out, tuple):
            out, dep_ret = out
        out = out.reshape(bsz, seq_len, dep_graph_len, hidden_size)
        if event_mask is not None:
            out = torch.where(event_mask[:, :, None, None], out, 0.0)
            present = dep_ret.get("present_key_value") if isinstance(dep_ret, dict) else None
            if present is not None and not bool(event_mask.all()):
                # the reference scatters the present keys / values of the kept events into zeros (:186-193)
                keep = event_mask.reshape(bsz * seq_len, 1, 1, 1)
                dep_ret["present_key_value"] = tuple(torch.where(keep, t, 0.0) for t in present)
        return out, {"seq_module": seq_ret, "dep_graph_module": dep_ret}
