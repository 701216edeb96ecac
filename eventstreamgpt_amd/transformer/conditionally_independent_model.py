"""Conditionally independent generative model — drop-in for
``EventStream/transformer/conditionally_independent_model.py`` (training path)."""
from __future__ import annotations

import torch

from .config import StructuredEventProcessingMode, StructuredTransformerConfig
from .model_output import GenerativeOutputLayerBase, GenerativeSequenceModelOutput, fused_ci_losses
from .transformer import ConditionallyIndependentPointProcessTransformer, StructuredTransformerPreTrainedModel


class ConditionallyIndependentGenerativeOutputLayer(GenerativeOutputLayerBase):
    """All event contents predicted from the shifted history encoding; TTE from the unshifted one
    (``conditionally_independent_model.py:24-161``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
            raise ValueError(f"{config.structured_event_processing_mode} invalid!")

    def forward(self, batch, encoded: torch.FloatTensor, is_generation: bool = False) -> GenerativeSequenceModelOutput:
        if is_generation:
            raise NotImplementedError("eventstreamgpt_amd: generation is out of scope for this build")
        losses, names = fused_ci_losses(self, batch, encoded)
        return self._package(batch, losses, names)


class CIPPTForGenerativeSequenceModeling(StructuredTransformerPreTrainedModel):
    """``CIPPTForGenerativeSequenceModeling`` (``:164-283``): encoder + output layer."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
            raise ValueError(f"{config.structured_event_processing_mode} invalid!")
        self.encoder = ConditionallyIndependentPointProcessTransformer(config)
        self.output_layer = ConditionallyIndependentGenerativeOutputLayer(config)
        self.post_init()

    def forward(self, batch, is_generation: bool = False, **kwargs) -> GenerativeSequenceModelOutput:
        encoded = self.encoder(batch, **kwargs)
        out = self.output_layer(batch, encoded.last_hidden_state, is_generation=is_generation)
        if kwargs.get("output_hidden_states", False):
            out["hidden_states"] = encoded.hidden_states
        return out
