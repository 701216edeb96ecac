"""Nested attention generative model — drop-in for ``EventStream/transformer/nested_attention_model.py``."""
from __future__ import annotations

import torch

from ..data.types import PytorchBatch
from .config import StructuredEventProcessingMode, StructuredTransformerConfig
from .generation.generation_utils import StructuredGenerationMixin
from .model_output import (
    GenerativeOutputLayerBase,
    GenerativeSequenceModelLabels,
    GenerativeSequenceModelLosses,
    GenerativeSequenceModelOutput,
    GenerativeSequenceModelPredictions,
    _level_sets,
    all_classification_measurements,
    all_regression_measurements,
    fused_na_losses,
)
from .transformer import (
    NestedAttentionPointProcessTransformer,
    StructuredTransformerPreTrainedModel,
    expand_mask,
    time_from_deltas,
)


class NestedAttentionGenerativeOutputLayer(GenerativeOutputLayerBase):
    """Level i of the dependency graph predicts its measurements from encoded[:, :, i-1]; TTE from the last
    (whole-event) level (``nested_attention_model.py:25-228``)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.NESTED_ATTENTION:
            raise ValueError(f"{config.structured_event_processing_mode} invalid for this model!")

    def forward(self, batch, encoded: torch.FloatTensor, is_generation: bool = False,
                dep_graph_el_generation_target: int | None = None) -> GenerativeSequenceModelOutput:
        if dep_graph_el_generation_target is not None and not is_generation:
            raise ValueError(
                f"If dep_graph_el_generation_target ({dep_graph_el_generation_target}) is not None, "
                f"is_generation ({is_generation}) must be True!"
            )
        if is_generation:
            return self._generation_output(batch, encoded, dep_graph_el_generation_target)
        losses, names = fused_na_losses(self, batch, encoded)
        return self._package(batch, losses, names)

    def _generation_output(self, batch, encoded, target):
        """``nested_attention_model.py:107-228`` with ``is_generation=True``: target None / 0 -> TTE only (from the
        whole-event level); target t > 0 -> the measurements of level t from encoded[:, :, t-1] (or from the only
        level when the encoder saw a single graph element)."""
        c = self.config
        G = encoded.shape[2]
        if target is None or target == 0:
            loop, do_tte = (), True
        else:
            loop, do_tte = ((1,) if G == 1 else (target,)), False
        cls_all = all_classification_measurements(self)
        reg_all = all_regression_measurements(c)
        cls, reg = {}, {}
        for i in loop:
            t_idx = target if target is not None else i
            cat, num = _level_sets(c.measurements_per_dep_graph_level[t_idx])
            cd, rd = self.generation_distributions(encoded[:, :, i - 1, :], cat & cls_all, num & reg_all)
            cls.update(cd)
            reg.update(rd)
        tte = self.TTE_layer(encoded[:, :, -1, :]) if do_tte else None
        return GenerativeSequenceModelOutput(
            loss=None,
            losses=GenerativeSequenceModelLosses(classification=None, regression=None, time_to_event=None),
            preds=GenerativeSequenceModelPredictions(classification=cls, regression=reg, regression_indices=None,
                                                     time_to_event=tte),
            labels=GenerativeSequenceModelLabels(classification=None, regression=None, regression_indices=None,
                                                 time_to_event=None),
            event_mask=batch["event_mask"],
            dynamic_values_mask=batch["dynamic_values_mask"],
        )


class NAPPTForGenerativeSequenceModeling(StructuredGenerationMixin, StructuredTransformerPreTrainedModel):
    """``NAPPTForGenerativeSequenceModeling`` (``:231-366``), with ``generate`` (with or without caches)."""

    def __init__(self, config: StructuredTransformerConfig):
        super().__init__(config)
        if config.structured_event_processing_mode != StructuredEventProcessingMode.NESTED_ATTENTION:
            raise ValueError(f"{config.structured_event_processing_mode} invalid for this model!")
        self.encoder = NestedAttentionPointProcessTransformer(config)
        self.output_layer = NestedAttentionGenerativeOutputLayer(config)
        self.post_init()

    def prepare_inputs_for_generation(self, batch: PytorchBatch, past=None, **kwargs) -> dict:
        """``nested_attention_model.py:265-324``: without a cache the batch as is; with one, the sequence key mask
        over the full batch and, once a past exists, absolute times from the deltas and the batch trimmed to its last
        event. ``past`` is ``{"seq_past": ..., "dep_graph_past": ...}`` as the encoder returns it."""
        if not kwargs.get("use_cache", False):
            return {**kwargs, "batch": batch}
        target = kwargs.get("dep_graph_el_generation_target", None)
        seq_attention_mask = expand_mask(batch.event_mask, batch.time_delta.dtype)
        if past is None:
            dep_graph_past = None
            if target is not None:
                raise ValueError(f"Can't have dep target {target} without past")
        elif isinstance(past, dict) and "seq_past" in past and "dep_graph_past" in past:
            dep_graph_past = past["dep_graph_past"]
            past = past["seq_past"]
            batch.time = time_from_deltas(batch)
            batch = batch.last_sequence_element_unsqueezed()
            if dep_graph_past is not None and target is None:
                raise ValueError("Trying to use generate with a past without a dep graph generation target!")
            if dep_graph_past is None and target is not None:
                raise ValueError("Trying to target only one dep graph element without past!")
        else:
            raise ValueError(f"{past} malformed!")
        return {**kwargs, "batch": batch, "past": past, "dep_graph_past": dep_graph_past,
                "seq_attention_mask": seq_attention_mask}

    def forward(self, batch, is_generation: bool = False, **kwargs) -> GenerativeSequenceModelOutput:
        encoded = self.encoder(batch, **kwargs)
        out = self.output_layer(batch, encoded.last_hidden_state, is_generation=is_generation,
                                dep_graph_el_generation_target=kwargs.get("dep_graph_el_generation_target", None))
        if kwargs.get("use_cache", False):
            out["past_key_values"] = encoded.past_key_values
        if kwargs.get("output_hidden_states", False):
            out["hidden_states"] = encoded.hidden_states
        return out
