"""Nested attention generative model — drop-in for ``EventStream/transformer/nested_attention_model.py``
(training path)."""
from __future__ import annotations

import torch

from .config import StructuredEventProcessingMode, StructuredTransformerConfig
from .model_output import GenerativeOutputLayerBase, GenerativeSequenceModelOutput, fused_na_losses
from .transformer import NestedAttentionPointProcessTransformer, StructuredTransformerPreTrainedModel


class NestedAttentionGenerativeOutputLayer(GenerativeOutputLayerBase):
    """Level i of the dependency graph predicts its measurements from encoded[:, :, i-1]; TTE from the last
    (whole-event) level (``nested_attention_model.py:25-228``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.NESTED_ATTENTION:
            raise ValueError(f"{config.structured_event_processing_mode} invalid for this model!")

    def forward(self, batch, encoded: torch.FloatTensor, is_generation: bool = False,
                dep_graph_el_generation_target: int | None = None) -> GenerativeSequenceModelOutput:
        if is_generation or dep_graph_el_generation_target is not None:
            raise NotImplementedError("eventstreamgpt_amd: generation is out of scope for this build")
        losses, names = fused_na_losses(self, batch, encoded)
        return self._package(batch, losses, names)


class NAPPTForGenerativeSequenceModeling(StructuredTransformerPreTrainedModel):
    """``NAPPTForGenerativeSequenceModeling`` (``:231-366``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.NESTED_ATTENTION:
            raise ValueError(f"{config.structured_event_processing_mode} invalid for this model!")
        self.encoder = NestedAttentionPointProcessTransformer(config)
        self.output_layer = NestedAttentionGenerativeOutputLayer(config)
        self.post_init()

    def forward(self, batch, is_generation: bool = False, **kwargs) -> GenerativeSequenceModelOutput:
        encoded = self.encoder(batch, **kwargs)
        out = self.output_layer(batch, encoded.last_hidden_state, is_generation=is_generation)
        if kwargs.get("output_hidden_states", False):
            out["hidden_states"] = encoded.hidden_states
        return out
