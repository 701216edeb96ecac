"""Stream classification on top of the event-stream encoder: the reference's fine-tuning model
(``EventStream/transformer/fine_tuning_model.py:15-91``, ``ESTForStreamClassification``) on this package's encoders,
so fine-tuning runs the same HIP hot path as pre-training.

The encoder's per-event states (the last dependency-graph level for nested-attention models) are pooled over the
sequence — ``cls`` (first position), ``last`` (last position, padding included, as the reference does), ``max`` /
``mean`` over the valid events (zero for a subject without any: ``safe_masked_max`` / ``safe_weighted_avg``,
``transformer/utils.py:61-207``) — and one Linear layer maps them to logits: a single logit with BCE-with-logits
when ``config.id2label == {0: False, 1: True}`` (string labels under transformers >= 5; then ``num_labels``
must be 2), else ``num_labels`` logits with
cross-entropy. Labels come from ``batch.stream_labels[config.finetuning_task]``.
"""
from __future__ import annotations

import torch

from ..data.types import PytorchBatch
from .config import StructuredEventProcessingMode, StructuredTransformerConfig
from .model_output import StreamClassificationModelOutput
from .transformer import (
    ConditionallyIndependentPointProcessTransformer,
    NestedAttentionPointProcessTransformer,
    StructuredTransformerPreTrainedModel,
)


def _valid(batch: PytorchBatch, like: torch.Tensor) -> torch.Tensor:
    """event_mask as [B, L, 1] in ``like``'s dtype / device."""
    return batch["event_mask"].to(device=like.device, dtype=like.dtype).unsqueeze(-1)


def _pool_max(x: torch.Tensor, batch: PytorchBatch) -> torch.Tensor:
    """Max over the valid events of x [B, L, D]; 0 for a subject without valid events."""
    m = torch.where(_valid(batch, x) > 0, x, torch.full_like(x, float("-inf"))).amax(dim=1)
    return torch.where(torch.isneginf(m), torch.zeros_like(m), m)


def _pool_mean(x: torch.Tensor, batch: PytorchBatch) -> torch.Tensor:
    """Mean over the valid events of x [B, L, D]; 0 for a subject without valid events."""
    w = _valid(batch, x)
    n = w.sum(dim=1)
    return torch.where(n > 0, (x * w).sum(dim=1) / torch.where(n > 0, n, torch.ones_like(n)), torch.zeros_like(n))


def _is_binary(id2label) -> bool:
    """The reference's ``config.id2label == {0: False, 1: True}``; transformers >= 5 only stores string labels, so
    {0: "False", 1: "True"} is the same declaration."""
    return id2label is not None and {int(k): str(v) for k, v in id2label.items()} == {0: "False", 1: "True"}


POOLING = {
    "cls": lambda x, batch: x[:, 0],
    "last": lambda x, batch: x[:, -1],
    "max": _pool_max,
    "mean": _pool_mean,
}


class ESTForStreamClassification(StructuredTransformerPreTrainedModel):
    """Fine-tuning model: encoder + pooling + logit layer + BCE / CE loss (``fine_tuning_model.py:15-91``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        self.task = config.finetuning_task
        encoder = (NestedAttentionPointProcessTransformer if self._uses_dep_graph
                   else ConditionallyIndependentPointProcessTransformer)
        self.encoder = encoder(config)
        self.pooling_method = config.task_specific_params["pooling_method"]
        binary = _is_binary(config.id2label)
        if binary:
            assert config.num_labels == 2
        self.logit_layer = torch.nn.Linear(config.hidden_size, 1 if binary else config.num_labels)
        self.criteria = torch.nn.BCEWithLogitsLoss() if binary else torch.nn.CrossEntropyLoss()
        self.post_init()

    @property
    def _uses_dep_graph(self) -> bool:
        return self.config.structured_event_processing_mode == StructuredEventProcessingMode.NESTED_ATTENTION

    def forward(self, batch: PytorchBatch, **kwargs) -> StreamClassificationModelOutput:
        hidden = self.encoder(batch, **kwargs).last_hidden_state
        if self._uses_dep_graph:
            hidden = hidden[:, :, -1, :]  # the last dependency-graph level summarises the event
        pool = POOLING.get(self.pooling_method)
        if pool is None:
            raise ValueError(f"{self.pooling_method} is not a supported pooling method.")
        logits = self.logit_layer(pool(hidden, batch)).squeeze(-1)
        labels = batch["stream_labels"][self.task]
        return StreamClassificationModelOutput(loss=self.criteria(logits, labels), preds=logits, labels=labels)
