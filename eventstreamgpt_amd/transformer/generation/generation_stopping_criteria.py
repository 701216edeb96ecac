"""Stopping criteria for event-stream generation (``transformer/generation/generation_stopping_criteria.py``)."""
from __future__ import annotations

from abc import ABC

from ...data.types import PytorchBatch


class StoppingCriteria(ABC):
    """``__call__(batch, outputs) -> bool``: True stops generation."""

    def __call__(self, batch: PytorchBatch, outputs, **kwargs) -> bool:
        raise NotImplementedError("StoppingCriteria needs to be subclassed")


class MaxLengthCriteria(StoppingCriteria):
    """Stops once the sequence (prompt included) holds ``max_length`` events."""

    def __init__(self, max_length: int):
        self.max_length = max_length

    def __call__(self, batch: PytorchBatch, outputs, **kwargs) -> bool:
        return batch.sequence_length >= self.max_length


class StoppingCriteriaList(list):
    def __call__(self, batch: PytorchBatch, outputs, **kwargs) -> bool:
        return any(criteria(batch, outputs) for criteria in self)
