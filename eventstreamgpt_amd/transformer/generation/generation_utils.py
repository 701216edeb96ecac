"""Autoregressive event-stream generation (``transformer/generation/generation_utils.py:73-416``).

``StructuredGenerationMixin.generate`` keeps the reference's arguments, checks and loop: expand the batch
``num_return_sequences`` times, then per generated event run the model on the (cache-trimmed) batch, slice the last
position's predictions, sample one event and append it (CI). With ``use_cache=True`` every layer keeps a
preallocated KV cache and the new event is attended by the decode kernel (``csrc/decode.hip``); the reference
re-concatenates its cache each step.

Host reads per generated event: one combined NaN / non-finite check over the inputs (the reference issues two
``.any()`` reads per input field), the sampler's own reads (data-dependent widths in ``strip_unused_indices``),
and the stopping criterion. The nested-attention model walks the dependency graph per event (target 0 = TTE and
the new event, then one graph level per call); with ``use_cache=True`` each call runs only the new event (target 0)
or the new graph element (t > 0) against the sequence and dependency-graph caches.
"""
from __future__ import annotations

import logging
import warnings
from dataclasses import dataclass
from typing import Any

import torch
import torch.distributed as dist
from transformers.utils import ModelOutput

from ...data.types import PytorchBatch
from ..config import StructuredEventProcessingMode
from .generation_stopping_criteria import MaxLengthCriteria, StoppingCriteriaList

logger = logging.getLogger(__name__)

_CHECKED_KEYS = ("dynamic_indices", "dynamic_values", "dynamic_measurement_indices", "time_delta", "time")


@dataclass
class SampleDecoderOnlyOutput(ModelOutput):
    """``generation_utils.py:40-70``: the generated batch plus optional per-step scores / attentions / states."""

    batch: PytorchBatch | None = None
    scores: tuple | None = None
    attentions: tuple | None = None
    hidden_states: tuple | None = None


def _check_finite(batch: PytorchBatch, generated_event_index: int) -> None:
    """The reference's per-field NaN then non-finite checks (``:237-262``), evaluated with one host read."""
    fields = [(k, batch[k]) for k in _CHECKED_KEYS if isinstance(batch[k], torch.Tensor)]
    if not fields:
        return
    counts = torch.stack([torch.stack([torch.isnan(v).sum(), (~torch.isfinite(v)).sum()]) for _, v in fields])
    counts = counts.tolist()
    for (k, _), (n_nan, n_nonfinite) in zip(fields, counts):
        if n_nan:
            raise ValueError(f"{n_nan} NaNs detected in {k} on index {generated_event_index}!")
        if n_nonfinite:
            raise ValueError(f"{n_nonfinite} Non-finites detected in {k} on index {generated_event_index}.")


class StructuredGenerationMixin:
    """Mixed into ``CIPPTForGenerativeSequenceModeling``; the model supplies ``prepare_inputs_for_generation``."""

    @staticmethod
    def _expand_inputs_for_generation(batch: PytorchBatch, expand_size: int = 1) -> PytorchBatch:
        return batch.repeat_batch_elements(expand_size)

    @staticmethod
    def _update_model_kwargs_for_generation(outputs: ModelOutput, model_kwargs: dict[str, Any]) -> dict[str, Any]:
        model_kwargs["past"] = outputs["past_key_values"] if "past_key_values" in outputs else None
        return model_kwargs

    def prepare_inputs_for_generation(self, batch: PytorchBatch, **kwargs) -> dict[str, Any]:
        raise NotImplementedError(
            "A model class needs to define a `prepare_inputs_for_generation` method in order to use `generate`."
        )

    def _get_stopping_criteria(self, max_length: int | None, stopping_criteria: StoppingCriteriaList | None):
        criteria = StoppingCriteriaList()
        if max_length is not None:
            criteria.append(MaxLengthCriteria(max_length=max_length))
        return self._merge_criteria_processor_list(criteria, stopping_criteria or StoppingCriteriaList())

    @staticmethod
    def _merge_criteria_processor_list(default_list, custom_list):
        if len(custom_list) == 0:
            return default_list
        for default in default_list:
            for custom in custom_list:
                if type(custom) is type(default):
                    raise ValueError(
                        f"A custom stopping criteria of type {type(custom)} with values {custom} has been passed to "
                        f"`generate`, but it has already been created with the values {default}."
                    )
        default_list.extend(custom_list)
        return default_list

    @torch.no_grad()
    def generate(self, batch: PytorchBatch, max_length: int | None = None, do_sample: bool | None = True,
                 num_return_sequences: int | None = None, max_new_events: int | None = None,
                 use_cache: bool | None = None, stopping_criteria: StoppingCriteriaList | None = None,
                 output_attentions: bool | None = None, output_hidden_states: bool | None = None,
                 output_scores: bool | None = None, return_dict_in_generate: bool | None = None,
                 synced_gpus: bool | None = False, **model_kwargs) -> SampleDecoderOnlyOutput | PytorchBatch:
        cfg = self.config
        do_sample = do_sample if do_sample is not None else getattr(cfg, "do_sample", True)
        if not do_sample:
            raise ValueError("Only `do_sample=True` mode is currently supported")
        num_return_sequences = (num_return_sequences if num_return_sequences is not None
                                else getattr(cfg, "num_return_sequences", 1))
        output_scores = output_scores if output_scores is not None else getattr(cfg, "output_scores", False)
        output_attentions = (output_attentions if output_attentions is not None
                             else getattr(cfg, "output_attentions", False))
        output_hidden_states = (output_hidden_states if output_hidden_states is not None
                                else getattr(cfg, "output_hidden_states", False))
        return_dict_in_generate = (return_dict_in_generate if return_dict_in_generate is not None
                                   else getattr(cfg, "return_dict_in_generate", False))
        model_kwargs["use_cache"] = use_cache
        model_kwargs["output_attentions"] = output_attentions
        model_kwargs["output_hidden_states"] = output_hidden_states

        if not bool(batch["event_mask"][:, -1].all()):
            logger.warning(
                "A decoder-only architecture is being used, but right-padding was detected! For correct generation "
                "results, please set `seq_padding_side='left'` when initializing the data."
            )
        input_seq_length = batch.sequence_length
        if max_length is None and max_new_events is None:
            warnings.warn(
                "Neither `max_length` nor `max_new_events` has been set, `max_length` will default to "
                f"{getattr(cfg, 'max_length', None)} (`self.config.max_length`).", UserWarning)
        elif max_length is None and max_new_events is not None:
            max_length = max_new_events + input_seq_length
        elif max_length is not None and max_new_events is not None:
            raise ValueError(
                "Both `max_new_events` and `max_length` have been set but they serve the same purpose -- setting a "
                "limit to the generated output length. Remove one of those arguments."
            )
        max_length = max_length if max_length is not None else getattr(cfg, "max_length", None)
        if max_length is not None:
            if input_seq_length >= max_length:
                logger.warning(f"Input length is {input_seq_length}, but `max_length` is set to {max_length}. This "
                               "can lead to unexpected behavior. You should consider increasing `max_new_events`.")
            if max_length > cfg.max_seq_len:
                raise ValueError("Can't run for a maximum length longer than the current maximum sequence length!")
        stopping_criteria = self._get_stopping_criteria(max_length=max_length, stopping_criteria=stopping_criteria)

        batch = self._expand_inputs_for_generation(batch, expand_size=num_return_sequences)
        mode = cfg.structured_event_processing_mode
        if mode == StructuredEventProcessingMode.CONDITIONALLY_INDEPENDENT:
            sample_fn = self._conditionally_independent_sample_event
        elif mode == StructuredEventProcessingMode.NESTED_ATTENTION:
            sample_fn = self._nested_attention_sample_event
        else:
            raise ValueError(f"Unsupported structured event processing mode: {mode}")

        scores = () if (return_dict_in_generate and output_scores) else None
        decoder_attentions = () if (return_dict_in_generate and output_attentions) else None
        decoder_hidden_states = () if (return_dict_in_generate and output_hidden_states) else None
        unfinished_sequences = batch["event_mask"].new_ones(batch.batch_size)
        this_peer_finished = False
        generated_event_index = 0
        while True:
            if synced_gpus:
                # All ranks keep stepping until every rank is done (generation_utils.py:237-250).
                flag = torch.tensor(0.0 if this_peer_finished else 1.0).to(batch.device)
                dist.all_reduce(flag, op=dist.ReduceOp.SUM)
                if flag.item() == 0.0:
                    break
            if synced_gpus and this_peer_finished:
                continue
            _check_finite(batch, generated_event_index)
            batch, step_scores, attentions, hidden_states, model_kwargs = sample_fn(batch, generated_event_index,
                                                                                     **model_kwargs)
            if return_dict_in_generate:
                if output_scores:
                    scores += (step_scores,)
                if output_attentions:
                    decoder_attentions += (attentions,)
                if output_hidden_states:
                    decoder_hidden_states += (hidden_states,)
            if unfinished_sequences.max() == 0 or stopping_criteria(batch, scores):
                if not synced_gpus:
                    break
                this_peer_finished = True
            generated_event_index += 1

        if return_dict_in_generate:
            return SampleDecoderOnlyOutput(scores=scores, batch=batch, attentions=decoder_attentions,
                                           hidden_states=decoder_hidden_states)
        return batch

    def _conditionally_independent_sample_event(self, batch: PytorchBatch, generated_event_index: int,
                                                **model_kwargs):
        """One CI step (``generation_utils.py:310-338``): forward, last-position predictions, sample, append the
        new event (TTE + functional-time measurements), then fill its contents."""
        model_inputs = self.prepare_inputs_for_generation(batch, **model_kwargs)
        outputs = self(**model_inputs, return_dict=True, is_generation=True)
        model_kwargs = self._update_model_kwargs_for_generation(outputs, model_kwargs)
        next_event_preds = outputs.preds.slice((slice(None), -1))
        next_event = next_event_preds.sample(batch.event_mask)
        batch = next_event.append_to_batch(batch, self.config)
        batch = next_event.update_last_event_data(batch, self.config)
        return batch, next_event_preds, outputs.attentions, outputs.hidden_states, model_kwargs

    def _nested_attention_sample_event(self, batch: PytorchBatch, generated_event_index: int, **model_kwargs):
        """One NA event (``generation_utils.py:340-416``): graph level 0 samples the TTE and appends the event, then
        each later level is predicted from the batch updated so far and written into the last event."""
        levels = [{"time"}, *self.config.measurements_per_dep_graph_level[1:]]
        is_first = generated_event_index == 0
        scores, attentions, hidden_states = (), (), ()
        for target, to_fill in enumerate(levels):
            if is_first and target == 0:
                target = None
            _check_finite(batch, generated_event_index)
            model_inputs = self.prepare_inputs_for_generation(batch, dep_graph_el_generation_target=target,
                                                              **model_kwargs)
            outputs = self(**model_inputs, return_dict=True, is_generation=True)
            model_kwargs = self._update_model_kwargs_for_generation(outputs, model_kwargs)
            preds = outputs.preds.slice((slice(None), -1))
            scores += (preds,)
            attentions += (outputs.attentions,)
            hidden_states += (outputs.hidden_states,)
            nxt = preds.sample(batch.event_mask)
            if to_fill == {"time"}:
                batch = nxt.append_to_batch(batch, self.config)
            else:
                batch = nxt.update_last_event_data(batch, self.config, measurements_to_fill=to_fill)
        return batch, scores, attentions, hidden_states, model_kwargs
