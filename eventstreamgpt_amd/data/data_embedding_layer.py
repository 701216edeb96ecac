"""``DataEmbeddingLayer`` — drop-in for ``EventStream/data/data_embedding_layer.py:55-708``.

Same constructor signature, validation errors, parameter names (``embed_layer.weight`` or
``categorical_embed_layer.weight`` / ``cat_proj`` / ``numerical_embed_layer.weight`` / ``num_proj``) and forward
contract (``forward(batch) -> [B, L, D]`` or ``[B, L, G, D]``). The compute runs in the gfx950 embedding-bag
kernels (``csrc/embed.hip``) through ``kernels.JointEmbedFn`` / ``SplitBagsFn``; the ``nn.EmbeddingBag`` modules
are kept only as parameter holders so state_dicts and initialisation (N(0,1), padding row 0) are unchanged.
"""
from __future__ import annotations

import torch

from .. import _lib as L
from .data_embedding_enums import (  # noqa: F401  (re-exported like the reference module)
    MEAS_INDEX_GROUP_T,
    EmbeddingMode,
    MeasIndexGroupOptions,
    StaticEmbeddingMode,
)
from .types import PytorchBatch


class DataEmbeddingLayer(torch.nn.Module):
    """Embeds a ``PytorchBatch``'s dynamic and static data (see the reference docstring, ``:55-198``)."""

    def __init__(
        self,
        n_total_embeddings: int,
        out_dim: int,
        static_embedding_mode: StaticEmbeddingMode,
        categorical_embedding_dim: int | None = None,
        numerical_embedding_dim: int | None = None,
        split_by_measurement_indices: list[list[MEAS_INDEX_GROUP_T]] | None = None,
        do_normalize_by_measurement_index: bool = False,
        static_weight: float = 1 / 2,
        dynamic_weight: float = 1 / 2,
        categorical_weight: float = 1 / 2,
        numerical_weight: float = 1 / 2,
    ):
        super().__init__()
        if type(out_dim) is not int:
            raise TypeError("`out_dim` must be an `int`.")
        if out_dim <= 0:
            raise ValueError("`out_dim` must be positive.")
        if type(n_total_embeddings) is not int:
            raise TypeError("`n_total_embeddings` must be an `int`.")
        if n_total_embeddings <= 0:
            raise ValueError("`n_total_embeddings` must be positive.")
        if static_embedding_mode not in StaticEmbeddingMode.values():
            raise TypeError(
                "`static_embedding_mode` must be a `StaticEmbeddingMode` enum member: "
                f"{StaticEmbeddingMode.values()}."
            )
        if (categorical_embedding_dim is not None) or (numerical_embedding_dim is not None):
            if (categorical_embedding_dim is None) or (numerical_embedding_dim is None):
                raise ValueError(
                    "If either `categorical_embedding_dim` or `numerical_embedding_dim` is not `None`, "
                    "then both must be not `None`."
                )
            for name, v in (("categorical_embedding_dim", categorical_embedding_dim),
                            ("numerical_embedding_dim", numerical_embedding_dim)):
                if type(v) is not int:
                    raise TypeError(f"`{name}` must be an `int`.")
                if v <= 0:
                    raise ValueError(f"`{name}` must be positive.")
        if split_by_measurement_indices is not None:
            for group in split_by_measurement_indices:
                if type(group) is not list:
                    raise TypeError("`split_by_measurement_indices` must be a list of lists.")
                for index in group:
                    if not isinstance(index, (int, tuple)):
                        raise TypeError(
                            "`split_by_measurement_indices` must be a list of lists of ints and/or tuples."
                        )
                    if type(index) is tuple:
                        if len(index) != 2:
                            raise ValueError("Each tuple in `split_by_measurement_indices` must have length 2.")
                        idx, mode = index
                        if type(idx) is not int:
                            raise TypeError(
                                "The first element of each tuple in each list of "
                                "`split_by_measurement_indices` must be an int."
                            )
                        if mode not in MeasIndexGroupOptions.values():
                            raise TypeError(
                                "The second element of each tuple in each sublist of "
                                "`split_by_measurement_indices` must be a member of the "
                                f"`MeasIndexGroupOptions` enum: {MeasIndexGroupOptions.values()}."
                            )

        self.out_dim = out_dim
        self.static_embedding_mode = static_embedding_mode
        self.split_by_measurement_indices = split_by_measurement_indices
        self.do_normalize_by_measurement_index = do_normalize_by_measurement_index
        self.static_weight = static_weight / (static_weight + dynamic_weight)
        self.dynamic_weight = dynamic_weight / (static_weight + dynamic_weight)
        self.categorical_weight = categorical_weight / (categorical_weight + numerical_weight)
        self.numerical_weight = numerical_weight / (categorical_weight + numerical_weight)
        self.n_total_embeddings = n_total_embeddings

        if categorical_embedding_dim is None and numerical_embedding_dim is None:
            self.embedding_mode = EmbeddingMode.JOINT
            self.embed_layer = torch.nn.EmbeddingBag(n_total_embeddings, out_dim, mode="sum", padding_idx=0)
        else:
            self.embedding_mode = EmbeddingMode.SPLIT_CATEGORICAL_NUMERICAL
            self.categorical_embed_layer = torch.nn.EmbeddingBag(
                n_total_embeddings, categorical_embedding_dim, mode="sum", padding_idx=0
            )
            self.cat_proj = torch.nn.Linear(categorical_embedding_dim, out_dim)
            self.numerical_embed_layer = torch.nn.EmbeddingBag(
                n_total_embeddings, numerical_embedding_dim, mode="sum", padding_idx=0
            )
            self.num_proj = torch.nn.Linear(numerical_embedding_dim, out_dim)
        self._buckets = []  # the operators' int[] buckets ([] = un-bucketed)
        self._group_error = None
        if split_by_measurement_indices:
            # The reference raises this in forward (_split_batch_into_measurement_index_buckets, :529-535), not at
            # construction; the message is kept and raised on the first embedding call.
            for i, g in enumerate(split_by_measurement_indices):
                if len(g) == 0 and i > 0:
                    self._group_error = (
                        f"Empty measurement index group: {g} at index {i}! Only the first (i=0) group can be empty "
                        "(in cases where there are no FUNCTIONAL_TIME_DEPENDENT measurements)."
                    )
                    break
            from ..kernels import buckets_list, buckets_struct

            self._buckets = buckets_list(buckets_struct(split_by_measurement_indices))

    @staticmethod
    def get_measurement_index_normalziation(measurement_indices: torch.Tensor) -> torch.Tensor:
        """Reference helper (``:314-349``), kept for API compatibility; the kernels compute it in registers."""
        eq = measurement_indices.unsqueeze(-1) == measurement_indices.unsqueeze(-2)
        vals = torch.where(measurement_indices == 0, 0.0, 1.0 / eq.sum(-1).float())
        s = vals.sum(-1, keepdim=True)
        return vals / torch.where(s == 0, torch.ones_like(s), s)

    # -------------------------------------------------------------------------------------------------------
    @property
    def n_levels(self) -> int:
        return len(self.split_by_measurement_indices) if self.split_by_measurement_indices else 1

    def _flags(self) -> int:
        f = 0
        if self.do_normalize_by_measurement_index:
            f |= L.EMB_NORMALIZE
        if self.static_embedding_mode == StaticEmbeddingMode.SUM_ALL:
            f |= L.EMB_STATIC
        return f

    def embed(self, batch: PytorchBatch, time_layer=None, cumsum: bool = False) -> torch.Tensor:
        """Fused input-layer embedding: data embedding (+ temporal encoding at level 0, + cumsum over levels),
        masked by ``event_mask``. Returns f32 [B, L, G, D]."""
        from ..kernels import EmbedSpec, embed_epilogue, joint_embed, split_bags

        if self._group_error is not None:
            raise ValueError(self._group_error)
        flags = self._flags()
        sin_div = cos_div = None
        post = 0
        if time_layer is not None:
            post |= L.EMB_TIME
            if batch.time is not None:
                post |= L.EMB_TIME_ABS
            sin_div, cos_div = time_layer.sin_div_term, time_layer.cos_div_term
        if cumsum:
            post |= L.EMB_CUMSUM
        G = self.n_levels
        static = bool(flags & L.EMB_STATIC)
        if self.embedding_mode == EmbeddingMode.JOINT:
            spec = EmbedSpec(flags | post, self.static_weight, self.dynamic_weight, self._buckets, G)
            return joint_embed(self.embed_layer.weight, batch, spec, sin_div, cos_div)
        # SPLIT: bags -> one GEMM with [cat_proj | num_proj] -> epilogue (time / cumsum / mask).
        dw = self.dynamic_weight if static else 1.0
        cat_scale = dw * self.categorical_weight
        num_scale = dw * self.numerical_weight
        static_scale = self.static_weight if static else 0.0
        spec = EmbedSpec(flags, self.static_weight, self.dynamic_weight, self._buckets, G)
        x = split_bags(self.categorical_embed_layer.weight, self.numerical_embed_layer.weight, batch, spec,
                       cat_scale, num_scale, static_scale)
        from ..fused import GEMM_DTYPES, compute_dtype, gemm_supported, linear_op
        from ..kernels import split_projection

        x2 = x.reshape(-1, x.shape[-1])
        dt = compute_dtype()
        D = self.cat_proj.weight.shape[0]
        if (x2.is_cuda and dt in GEMM_DTYPES and gemm_supported(x2.shape[0], x2.shape[1], D)
                and self.cat_proj.bias is not None and self.num_proj.bias is not None):
            # projection + epilogue in one autograd node: no weight cat, bias arithmetic or dtype casts as
            # framework kernels (kernels._SplitProjection)
            return split_projection(x2, self.cat_proj, self.num_proj, cat_scale + static_scale, num_scale, batch, G,
                                    post, sin_div, cos_div, dt)
        w = torch.cat([self.cat_proj.weight, self.num_proj.weight], dim=1)
        bias = (cat_scale + static_scale) * self.cat_proj.bias + num_scale * self.num_proj.bias
        if x2.is_cuda and dt in GEMM_DTYPES and gemm_supported(x2.shape[0], w.shape[1], w.shape[0]):
            # the HIP GEMM, bf16 or exact f32 (bias in the epilogue; dW, db in one grouped backward launch)
            with torch.autocast("cuda", enabled=False):
                y = linear_op(x2.to(dt).contiguous(), w.detach().to(dt).contiguous(),
                              bias.float().contiguous(), [w]).float().view(*x.shape[:-1], w.shape[0])
        else:
            y = torch.nn.functional.linear(x, w, bias).float()
        return embed_epilogue(y, batch, G, post, sin_div, cos_div)

    def forward(self, batch: PytorchBatch) -> torch.Tensor:
        """``DataEmbeddingLayer.forward`` (``:609-708``): [B, L, D] or [B, L, G, D] (no temporal encoding)."""
        out = self.embed(batch)
        return out if self.split_by_measurement_indices else out.squeeze(2)
