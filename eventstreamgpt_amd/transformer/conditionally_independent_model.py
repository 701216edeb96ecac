"""Conditionally independent generative model — drop-in for
``EventStream/transformer/conditionally_independent_model.py`` (training path)."""
from __future__ import annotations

import torch

from .config import StructuredEventProcessingMode, StructuredTransformerConfig
from ..data.types import PytorchBatch
from .generation.generation_utils import StructuredGenerationMixin
from .model_output import (
    GenerativeOutputLayerBase,
    GenerativeSequenceModelLabels,
    GenerativeSequenceModelLosses,
    GenerativeSequenceModelOutput,
    fused_ci_losses,
)
from .transformer import (
    ConditionallyIndependentPointProcessTransformer,
    StructuredTransformerPreTrainedModel,
    expand_mask,
    time_from_deltas,
)


class ConditionallyIndependentGenerativeOutputLayer(GenerativeOutputLayerBase):
    """All event contents predicted from the shifted history encoding; TTE from the unshifted one
    (``conditionally_independent_model.py:24-161``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
            raise ValueError(f"{config.structured_event_processing_mode} invalid!")

    def forward(self, batch, encoded: torch.FloatTensor, is_generation: bool = False) -> GenerativeSequenceModelOutput:
        if is_generation:
            # Contents AND TTE from the unshifted encoding (conditionally_independent_model.py:88-89).
            return GenerativeSequenceModelOutput(
                loss=None,
                losses=GenerativeSequenceModelLosses(classification={}, regression={}, time_to_event=None),
                preds=self.generation_predictions(encoded),
                labels=GenerativeSequenceModelLabels(classification={}, regression={}, regression_indices={},
                                                     time_to_event=None),
                event_mask=batch["event_mask"],
                dynamic_values_mask=batch["dynamic_values_mask"],
            )
        losses, names = fused_ci_losses(self, batch, encoded)
        return self._package(batch, losses, names)


class CIPPTForGenerativeSequenceModeling(StructuredGenerationMixin, StructuredTransformerPreTrainedModel):
    """``CIPPTForGenerativeSequenceModeling`` (``:164-283``): encoder + output layer, and ``generate``."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
            raise ValueError(f"{config.structured_event_processing_mode} invalid!")
        self.encoder = ConditionallyIndependentPointProcessTransformer(config)
        self.output_layer = ConditionallyIndependentGenerativeOutputLayer(config)
        self.post_init()

    def prepare_inputs_for_generation(self, batch: PytorchBatch, past: tuple | None = None, **kwargs) -> dict:
        """``conditionally_independent_model.py:198-248``: absolute times from the deltas; with a cache, the key
        mask over the full sequence and the batch trimmed to its last event."""
        batch.time = time_from_deltas(batch)
        if not kwargs.get("use_cache", False):
            return {**kwargs, "batch": batch}
        seq_attention_mask = expand_mask(batch.event_mask, batch.time_delta.dtype)
        target = kwargs.get("dep_graph_el_generation_target", None)
        if target is not None:
            raise ValueError(f"Can't use dep_graph_el_generation_target ({target}) in a conditionally independent "
                             "model.")
        if past is None:
            pass
        elif isinstance(past, tuple):
            batch = batch.last_sequence_element_unsqueezed()
        else:
            raise ValueError(f"{past} malformed!")
        return {**kwargs, "seq_attention_mask": seq_attention_mask, "batch": batch, "past": past}

    def forward(self, batch, is_generation: bool = False, **kwargs) -> GenerativeSequenceModelOutput:
        encoded = self.encoder(batch, **kwargs)
        out = self.output_layer(batch, encoded.last_hidden_state, is_generation=is_generation)
        if kwargs.get("use_cache", False):
            out["past_key_values"] = encoded.past_key_values
        if kwargs.get("output_hidden_states", False):
            out["hidden_states"] = encoded.hidden_states
        return out
