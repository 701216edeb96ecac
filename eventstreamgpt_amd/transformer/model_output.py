"""Output containers and the fused generative output layer (``EventStream/transformer/model_output.py``).

``GenerativeOutputLayerBase`` keeps the reference's submodules and parameter names (``TTE_layer``,
``IsObservedLayer``, ``ClassificationLayer``, ``regression_layers``; ``:1253-1309``). Training losses follow
``get_TTE_outputs`` / ``get_classification_outputs`` / ``get_regression_outputs`` (``:1311-1721``) but are
computed by ONE head GEMM (all heads' weights concatenated along the output dimension) plus the fused loss kernel
(``kernels.output_loss``: ``torch.ops.esgpt.output_loss``), which also produces d(loss)/d(logits).

Head column layout of the fused GEMM: [ClassificationLayer (V) | IsObservedLayer (n_meas) |
regression_layers[m].proj (in measurements_per_generative_mode order) || TTE_layer.proj].
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from transformers.utils import ModelOutput

from .. import _lib as L
from ..data.data_embedding_enums import MeasIndexGroupOptions
from ..data.types import DataModality, PytorchBatch, TemporalityType
from ..fused import head_losses, linear_bias
from ..kernels import output_loss
from .config import TimeToEventGenerationHeadType
from .generative_layers import (
    ExponentialTTELayer,
    GaussianIndexedRegressionLayer,
    GaussianRegressionLayer,
    LogNormalMixtureDistribution,
    LogNormalMixtureTTELayer,
)


@dataclass
class TransformerOutputWithPast(ModelOutput):
    last_hidden_state: torch.FloatTensor = None
    past_key_values: tuple | dict | None = None
    hidden_states: tuple | None = None
    attentions: tuple | dict | None = None


@dataclass
class StreamClassificationModelOutput(ModelOutput):
    """Output of the stream classification (fine-tuning) model (``model_output.py:1220-1231``): the loss, the
    predictions (logits) and the labels."""

    loss: torch.FloatTensor
    preds: torch.FloatTensor = None
    labels: torch.LongTensor | torch.FloatTensor = None


@dataclass
class GenerativeSequenceModelLosses(ModelOutput):
    classification: dict[str, torch.FloatTensor] | None = None
    regression: dict[str, torch.FloatTensor] | None = None
    time_to_event: torch.FloatTensor | None = None


def _slice_value(val, idx):
    """``NestedIndexableMixin._recursive_slice`` (``model_output.py:181-193``) over the distribution types the heads
    build (the reference's ``idx_distribution``, ``utils.py:247``): parameters are indexed, event dims untouched."""
    D = torch.distributions
    if val is None:
        return None
    if isinstance(val, dict):
        return {k: _slice_value(v, idx) for k, v in val.items()}
    if isinstance(val, tuple):
        return tuple(_slice_value(v, idx) for v in val)
    if isinstance(val, LogNormalMixtureDistribution):
        locs, log_scales, log_weights = val.params
        return LogNormalMixtureDistribution(locs[idx], log_scales[idx], log_weights[idx], val.mean_log_inter_time,
                                            val.std_log_inter_time)
    if isinstance(val, D.Bernoulli):
        return D.Bernoulli(logits=val.logits[idx], validate_args=False)
    if isinstance(val, D.Categorical):
        return D.Categorical(logits=val.logits[idx], validate_args=False)
    if isinstance(val, D.Normal):
        return D.Normal(loc=val.loc[idx], scale=val.scale[idx], validate_args=False)
    if isinstance(val, D.Exponential):
        return D.Exponential(rate=val.rate[idx], validate_args=False)
    if isinstance(val, D.Distribution):
        raise IndexError(f"eventstreamgpt_amd: cannot slice distribution {type(val).__name__}")
    return val[idx]


def strip_unused_indices(dynamic_indices, *other_tensors, width: int | None = None):
    """Moves the non-zero entries of ``dynamic_indices`` to the front of the last dim (stable) and trims it to the
    largest per-row count; ``other_tensors`` follow the same permutation, zero-filled (``model_output.py:108-169``).
    The output width is data-dependent: one host read unless the caller passes it (``width``)."""
    present = dynamic_indices != 0
    n = present.sum(-1)
    if width is None:
        width = int(n.max()) if n.numel() else 0
    order = torch.argsort((~present).to(torch.int8), dim=-1, stable=True)[..., :width]
    keep = torch.arange(width, device=dynamic_indices.device) < n.unsqueeze(-1)

    def idx_fn(T):
        return torch.where(keep, torch.gather(T, -1, order), torch.zeros((), dtype=T.dtype, device=T.device))

    if not other_tensors:
        return idx_fn(dynamic_indices)
    return tuple([idx_fn(dynamic_indices), *[idx_fn(T) for T in other_tensors]])


def expand_indexed_regression(X: torch.Tensor, idx: torch.Tensor, vocab_size: int):
    """Dense [..., vocab_size] with X scattered at idx (``utils.py:33-58``)."""
    expanded = torch.zeros(*idx.shape[:-1], vocab_size, device=X.device, dtype=X.dtype)
    return expanded.scatter(-1, idx, X)


def _ordered(config, measurements):
    """Deterministic iteration over a measurement set (the reference iterates a python set, whose order varies
    with hash seeding): measurement index order, event_type first; (name, group) tuples by name."""
    def key(m):
        name = m[0] if isinstance(m, (list, tuple)) else m
        return (config.measurements_idxmap.get(name, 1 << 30), str(m))

    return sorted(measurements, key=key)


@dataclass
class GenerativeSequenceModelSamples(ModelOutput):
    """One sampled next event per subject (``model_output.py:247-1072``): event_mask [B], time_to_event [B],
    classification {m: [B] labels (single) | [B, vocab] 0/1 (multi)}, regression {m: [B, n] | [B, 1] (NaN =
    unobserved)}, regression_indices."""

    event_mask: torch.BoolTensor | None = None
    time_to_event: torch.FloatTensor | None = None
    classification: dict | None = None
    regression: dict | None = None
    regression_indices: dict | None = None

    def _build_new_batch_element(self, batch: PytorchBatch, config):
        """(time_delta, event_mask, indices, meas, values, values_mask) of the appended event: only functional
        time-dependent measurements are filled here (``:279-390``)."""
        di, dm, dv, dvm = [], [], [], []
        event_mask = self.event_mask
        new_time = None
        for m, cfg in (config.measurement_configs or {}).items():
            if getattr(cfg, "temporality", None) != TemporalityType.FUNCTIONAL_TIME_DEPENDENT:
                continue
            if getattr(cfg, "modality", None) == DataModality.DROPPED:
                continue
            if new_time is None:
                duration = torch.where(batch.event_mask[:, :-1], batch.time_delta[:, :-1], 0).sum(-1)
                new_time = torch.where(event_mask, batch.start_time + duration + self.time_to_event, 0)
            mi = config.measurements_idxmap[m]
            is_meas = batch.dynamic_measurement_indices[:, -1, :] == mi
            indices = torch.where(is_meas, batch.dynamic_indices[:, -1, :], 0).sum(-1)
            vals = torch.where(is_meas & batch.dynamic_values_mask[:, -1, :], batch.dynamic_values[:, -1, :],
                               0).sum(-1)
            offset = config.vocab_offsets_by_measurement[m]
            new_indices, new_values = cfg.functor.update_from_prior_timepoint(
                prior_indices=indices - offset, prior_values=vals, new_delta=self.time_to_event, new_time=new_time,
                vocab=cfg.vocabulary, measurement_metadata=cfg.measurement_metadata)
            new_indices = (new_indices + offset).unsqueeze(-1)
            new_values = new_values.unsqueeze(-1)
            di.append(new_indices)
            dvm.append(~torch.isnan(new_values))
            dv.append(torch.nan_to_num(new_values, nan=0, posinf=0, neginf=0))
            dm.append(mi * torch.ones_like(new_indices))
        if di:
            cat = [torch.cat(x, 1) for x in (di, dm, dv, dvm)]
        else:
            # The reference builds [B, 1, 0] (CI) / [B, 1, G, 0] (NA) here; its strip_unused_indices indexes rows
            # along dim 0 only, so both come out as [B, 0].
            z = torch.zeros(batch.batch_size, 0, dtype=torch.long, device=batch.device)
            cat = [z, torch.zeros_like(z), torch.zeros_like(z).float(), torch.zeros_like(z).bool()]
        if not di:  # nothing to compact: skip the width read
            return (self.time_to_event, event_mask, *cat)
        return (self.time_to_event, event_mask, *strip_unused_indices(*cat))

    def format_updates_to_last_batch_event(self, batch: PytorchBatch, config, measurements_to_build=None):
        """Sampled contents of ``measurements_to_build`` as (indices, meas, values, values_mask) [B, n]
        (``:392-616``)."""
        raw, bad = self._format_updates_raw(batch, config, measurements_to_build)
        if bad is not None and bool(bad.any()):
            raise ValueError("For {measurement}, need preds < vocab_size!")
        return strip_unused_indices(*raw)

    def _format_updates_raw(self, batch: PytorchBatch, config, measurements_to_build):
        """The updates before the final compaction, plus a device flag of out-of-range single-label samples (the
        reference raises on them; the caller reads the flag with its other host reads). The reference compacts
        each multi-label block on the way too; the final stable compaction gives the same result without those
        host reads."""
        di, dm, dv, dvm = [], [], [], []
        bad = []

        def zeros_like_last():
            dv.append((0 * di[-1]).float())
            dvm.append((0 * di[-1]).bool())

        def add_single(m):
            if m not in config.vocab_offsets_by_measurement:
                raise ValueError(f"Missing {m}")
            off = config.vocab_offsets_by_measurement[m]
            size = config.vocab_sizes_by_measurement[m]
            if m not in self.classification:
                print(f"WARNING: Attempting to generate improper measurement {m}! "
                      f"Acceptable targets: {', '.join(self.classification.keys())}")
                return False
            preds = self.classification[m]
            if len(preds.shape) != 1:
                raise ValueError(f"For {m}, expect 1D preds, got {preds.shape}!")
            bad.append((preds >= size).any())
            idx = off + preds
            di.append(idx.unsqueeze(-1))
            dm.append((config.measurements_idxmap[m] * torch.ones_like(idx)).unsqueeze(-1))
            return True

        def add_multi(m):
            if m not in config.vocab_offsets_by_measurement:
                raise ValueError(f"Missing {m}")
            off = config.vocab_offsets_by_measurement[m]
            size = config.vocab_sizes_by_measurement[m]
            if m not in self.classification:
                print(f"WARNING: Attempting to generate improper measurement {m}!")
                return False
            preds = self.classification[m]
            if len(preds.shape) != 2:
                raise ValueError(f"For {m}, expect 2D preds, got {preds.shape}!")
            if preds.shape[-1] != size:
                raise ValueError(f"For {m}, expect preds.shape[-1] == vocab_size, got {preds.shape[-1]}!")
            idx = (torch.arange(size, device=preds.device).long() + off).unsqueeze(0).expand_as(preds)
            idx = torch.where(preds == 1, idx, 0)
            di.append(idx)
            dm.append(config.measurements_idxmap[m] * (idx != 0).long())
            return True

        def add_univariate(m):
            if m not in self.regression:
                raise ValueError(f"Attempting to generate improper measurement {m}!")
            preds = self.regression[m].squeeze(-1)
            if len(preds.squeeze(-1).shape) != 1:
                raise ValueError(f"For {m}, expect 1D preds, got {preds.shape}!")
            dvm.append(~torch.isnan(preds.unsqueeze(-1)))
            dv.append(torch.nan_to_num(preds.unsqueeze(-1), nan=0))

        def add_multivariate(m, indices):
            if m not in self.regression:
                raise ValueError(f"Attempting to generate improper measurement {m}!")
            vals = self.regression[m]
            vmask = torch.ones_like(vals).bool()
            size = config.vocab_sizes_by_measurement[m]
            ri = self.regression_indices
            if ri is not None and m in ri and ri[m] is not None:
                vals = expand_indexed_regression(vals, ri[m], size)
                vmask = expand_indexed_regression(vmask, ri[m], size)
            off = config.vocab_offsets_by_measurement[m]
            mask = indices >= off
            gidx = torch.where(mask, indices - off, 0).long()
            dv.append(torch.where(mask, vals.gather(-1, gidx), 0))
            dvm.append(torch.where(mask, vmask.gather(-1, gidx), False))

        if "event_type" in measurements_to_build:
            if add_single("event_type"):
                zeros_like_last()
        for m in _ordered(config, measurements_to_build):
            if type(m) in (list, tuple):
                assert len(m) == 2
                m, group_mode = m
            else:
                group_mode = None
            if m == "event_type":
                continue
            modality = config.measurement_configs[m].modality
            if modality == DataModality.SINGLE_LABEL_CLASSIFICATION and group_mode is None:
                if add_single(m):
                    zeros_like_last()
            elif modality == DataModality.MULTI_LABEL_CLASSIFICATION and group_mode is None:
                if add_multi(m):
                    zeros_like_last()
            elif modality == DataModality.UNIVARIATE_REGRESSION and group_mode is None:
                add_univariate(m)
                di.append(config.vocab_offsets_by_measurement[m] * dvm[-1].long())
                dm.append(config.measurements_idxmap[m] * dvm[-1].long())
            elif modality == DataModality.MULTIVARIATE_REGRESSION and group_mode in (
                    None, MeasIndexGroupOptions.CATEGORICAL_AND_NUMERICAL):
                if add_multi(m):
                    add_multivariate(m, indices=di[-1])
            elif modality == DataModality.MULTIVARIATE_REGRESSION and group_mode == MeasIndexGroupOptions.CATEGORICAL_ONLY:
                if add_multi(m):
                    zeros_like_last()
            elif modality == DataModality.MULTIVARIATE_REGRESSION and group_mode == MeasIndexGroupOptions.NUMERICAL_ONLY:
                mi = config.measurements_idxmap[m]
                existing = batch.dynamic_measurement_indices[:, -1] == mi
                idx = torch.where(existing, batch.dynamic_indices[:, -1], 0)
                di.append(idx)
                dm.append(mi * torch.ones_like(idx))
                add_multivariate(m, indices=idx)
            else:
                raise ValueError(f"{modality}, {group_mode} invalid!")
        raw = (torch.cat(di, 1), torch.cat(dm, 1), torch.cat(dv, 1), torch.cat(dvm, 1))
        return raw, (torch.stack(bad) if bad else None)

    @staticmethod
    def pad_data_elements(batch: PytorchBatch, new_di, new_dm, new_dv, new_dvm):
        """Right-pads either the batch's or the new event's data-element dim to the wider of the two
        (``:619-860``)."""
        di, dm, dv, dvm = (batch.dynamic_indices, batch.dynamic_measurement_indices, batch.dynamic_values,
                           batch.dynamic_values_mask)
        n_old, n_new = di.shape[-1], new_di.shape[-1]
        pad = torch.nn.functional.pad
        if n_new < n_old:
            d = n_old - n_new
            new_di, new_dm, new_dv = pad(new_di, (0, d), value=0), pad(new_dm, (0, d), value=0), pad(new_dv, (0, d),
                                                                                                     value=0)
            new_dvm = pad(new_dvm, (0, d), value=False)
        elif n_new > n_old:
            d = n_new - n_old
            di, dm, dv = pad(di, (0, d), value=0), pad(dm, (0, d), value=0), pad(dv, (0, d), value=0)
            dvm = pad(dvm, (0, d), value=False)
        return (di, dm, dv, dvm), (new_di, new_dm, new_dv, new_dvm)

    def append_to_batch(self, batch: PytorchBatch, config) -> PytorchBatch:
        """Sets the last event's time_delta to the sampled TTE and appends a new event (time_delta 1, mask copied
        from the last event, functional-time measurements filled) (``:862-942``)."""
        tte, emask, ndi, ndm, ndv, ndvm = self._build_new_batch_element(batch, config)
        time_delta = batch.time_delta.clone()
        time_delta[:, -1] = tte
        time_delta = torch.cat((time_delta, torch.ones_like(tte).unsqueeze(1)), 1)
        event_mask = torch.cat((batch.event_mask, emask.unsqueeze(1)), 1)
        (di, dm, dv, dvm), (ndi, ndm, ndv, ndvm) = self.pad_data_elements(batch, ndi, ndm, ndv, ndvm)
        return PytorchBatch(
            time_delta=time_delta, event_mask=event_mask,
            dynamic_indices=torch.cat((di, ndi.unsqueeze(1)), 1),
            dynamic_measurement_indices=torch.cat((dm, ndm.unsqueeze(1)), 1),
            dynamic_values=torch.cat((dv, ndv.unsqueeze(1)), 1),
            dynamic_values_mask=torch.cat((dvm, ndvm.unsqueeze(1)), 1),
            static_indices=batch.static_indices, static_measurement_indices=batch.static_measurement_indices,
            start_time=batch.start_time, stream_labels=batch.stream_labels, start_idx=batch.start_idx,
            end_idx=batch.end_idx, subject_id=batch.subject_id,
        )

    def update_last_event_data(self, batch: PytorchBatch, config, measurements_to_fill=None) -> PytorchBatch:
        """Writes the sampled contents into the last event, keeping its existing elements (minus NUMERICAL_ONLY
        measurements being re-filled) (``:944-1070``)."""
        if measurements_to_fill is None:
            measurements_to_fill = ["event_type"]
            for m, cfg in (config.measurement_configs or {}).items():
                if not cfg.is_dropped and cfg.temporality == TemporalityType.DYNAMIC:
                    measurements_to_fill.append(m)
            measurements_to_fill = set(measurements_to_fill)
        if not measurements_to_fill:
            return batch
        if "time" in measurements_to_fill:
            raise ValueError("You shouldn't ever be trying to fill the 'time' aspect of a batch!")
        prev = (batch.dynamic_indices[:, -1], batch.dynamic_measurement_indices[:, -1], batch.dynamic_values[:, -1],
                batch.dynamic_values_mask[:, -1])
        raw, bad = self._format_updates_raw(batch, config, measurements_to_fill)
        drop = torch.zeros_like(prev[0], dtype=torch.bool)
        for m in measurements_to_fill:
            if type(m) is not tuple or m[1] != MeasIndexGroupOptions.NUMERICAL_ONLY:
                continue
            drop |= prev[1] == config.measurements_idxmap[m[0]]
        prev = [torch.where(drop, 0, t) for t in prev]
        # ONE host read: both compacted widths and the out-of-range flag
        flags = [(prev[0] != 0).sum(-1).max(), (raw[0] != 0).sum(-1).max()]
        if bad is not None:
            flags.append(bad.any().long())
        read = torch.stack([f.long() for f in flags]).tolist()
        if bad is not None and read[2]:
            raise ValueError("For {measurement}, need preds < vocab_size!")
        prev = strip_unused_indices(*prev, width=read[0])
        new = strip_unused_indices(*raw, width=read[1])
        new = [torch.cat((p, n), 1) for p, n in zip(prev, new)]
        (di, dm, dv, dvm), (ndi, ndm, ndv, ndvm) = self.pad_data_elements(batch, *new)
        di, dm, dv, dvm = di.clone(), dm.clone(), dv.clone(), dvm.clone()
        di[:, -1], dm[:, -1], dv[:, -1], dvm[:, -1] = ndi, ndm, ndv, ndvm
        return PytorchBatch(
            time_delta=batch.time_delta, event_mask=batch.event_mask, dynamic_indices=di,
            dynamic_measurement_indices=dm, dynamic_values=dv, dynamic_values_mask=dvm,
            static_indices=batch.static_indices, static_measurement_indices=batch.static_measurement_indices,
            start_time=batch.start_time, stream_labels=batch.stream_labels, start_idx=batch.start_idx,
            end_idx=batch.end_idx, subject_id=batch.subject_id,
        )


@dataclass
class GenerativeSequenceModelPredictions(ModelOutput):
    classification: dict | None = None
    regression: dict | None = None
    regression_indices: dict | None = None
    time_to_event: torch.distributions.Distribution | None = None

    def slice(self, idx):
        """Every prediction indexed by ``idx`` over its batch dims (``NestedIndexableMixin.slice``, ``:195-205``)."""
        return self.__class__(classification=_slice_value(self.classification, idx),
                              regression=_slice_value(self.regression, idx),
                              regression_indices=_slice_value(self.regression_indices, idx),
                              time_to_event=_slice_value(self.time_to_event, idx))

    def sample(self, event_mask: torch.BoolTensor) -> GenerativeSequenceModelSamples:
        """Draws one event from the predictions (``model_output.py:1093-1166``), in the reference's draw order per
        measurement (is-observed first, then the value)."""
        D = torch.distributions
        cls = None
        if self.classification is not None:
            if not isinstance(self.classification, dict):
                raise ValueError(f"self.classification is malformed! Got\n{self.classification}")
            cls = {}
            for k, v in self.classification.items():
                if isinstance(v, tuple) and len(v) == 2 and v[0] is None and isinstance(v[1], D.Bernoulli):
                    cls[k] = v[1].sample()
                elif (isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], D.Bernoulli)
                      and isinstance(v[1], D.Categorical)):
                    is_obs = v[0].sample() == 1
                    samp = v[1].sample()
                    cls[k] = torch.where(is_obs, samp, torch.zeros_like(samp))
                else:
                    raise ValueError(f"Don't know how to sample classification dist {v}!")
        reg = None
        if self.regression is not None:
            if not isinstance(self.regression, dict):
                raise ValueError(f"self.regression is malformed! Got\n{self.regression}")
            reg = {}
            for k, v in self.regression.items():
                if isinstance(v, tuple) and len(v) == 2 and v[0] is None and isinstance(v[1], D.Normal):
                    reg[k] = v[1].sample()
                elif (isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], D.Bernoulli)
                      and isinstance(v[1], D.Normal)):
                    is_obs = v[0].sample() == 1
                    samp = v[1].sample()
                    is_obs = is_obs.unsqueeze(-1).expand_as(samp)
                    reg[k] = torch.where(is_obs, samp, float("nan") * torch.ones_like(samp))
                else:
                    raise ValueError(f"Don't know how to sample regression dist {v}!")
        tte = None
        if self.time_to_event is not None:
            tte = torch.nan_to_num(self.time_to_event.sample(), nan=None, posinf=1000)
        return GenerativeSequenceModelSamples(event_mask=event_mask[:, -1].detach(), classification=cls,
                                              regression=reg, regression_indices=self.regression_indices,
                                              time_to_event=tte)


@dataclass
class GenerativeSequenceModelLabels(ModelOutput):
    classification: dict | None = None
    regression: dict | None = None
    regression_indices: dict | None = None
    time_to_event: torch.FloatTensor | None = None


@dataclass
class GenerativeSequenceModelOutput(ModelOutput):
    loss: torch.FloatTensor = None
    losses: GenerativeSequenceModelLosses | None = None
    preds: GenerativeSequenceModelPredictions | None = None
    labels: GenerativeSequenceModelLabels | None = None
    event_mask: torch.BoolTensor | None = None
    dynamic_values_mask: torch.BoolTensor | None = None
    past_key_values: tuple | None = None
    hidden_states: tuple | None = None
    attentions: tuple | None = None


def _level_sets(level_spec):
    cat, num = set(), set()
    for m in level_spec:
        if isinstance(m, (tuple, list)):
            name, mode = m[0], str(m[1])
        else:
            name, mode = m, MeasIndexGroupOptions.CATEGORICAL_AND_NUMERICAL.value
        if mode in ("categorical_and_numerical", "categorical_only"):
            cat.add(name)
        if mode in ("categorical_and_numerical", "numerical_only"):
            num.add(name)
        if mode not in ("categorical_and_numerical", "categorical_only", "numerical_only"):
            raise ValueError(f"Unknown mode {mode}")
    return cat, num


class GenerativeOutputLayerBase(torch.nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        tte = config.TTE_generation_layer_type
        if tte == TimeToEventGenerationHeadType.LOG_NORMAL_MIXTURE:
            self.TTE_layer = LogNormalMixtureTTELayer(
                in_dim=config.hidden_size, num_components=config.TTE_lognormal_generation_num_components,
                mean_log_inter_time=config.mean_log_inter_event_time_min,
                std_log_inter_time=config.std_log_inter_event_time_min,
            )
        elif tte == TimeToEventGenerationHeadType.EXPONENTIAL:
            self.TTE_layer = ExponentialTTELayer(in_dim=config.hidden_size)
        else:
            raise ValueError(
                "Invalid option for `config.TTE_generation_layer_type`. Must be a member of the "
                f"`TimeToEventGenerationHeadType` enum: ({TimeToEventGenerationHeadType.values()}). got {tte}."
            )
        self.IsObservedLayer = torch.nn.Linear(config.hidden_size, len(config.measurements_idxmap))
        self.ClassificationLayer = torch.nn.Linear(config.hidden_size, config.vocab_size)
        self.regression_layers = torch.nn.ModuleDict({})
        for m in config.measurements_for(DataModality.MULTIVARIATE_REGRESSION):
            self.regression_layers[m] = GaussianIndexedRegressionLayer(
                n_regression_targets=config.vocab_sizes_by_measurement[m], in_dim=config.hidden_size)
        for m in config.measurements_for(DataModality.UNIVARIATE_REGRESSION):
            if m in self.regression_layers:
                raise ValueError(f"{m} duplicated!")
            self.regression_layers[m] = GaussianRegressionLayer(in_dim=config.hidden_size)
        self.classification_mode_per_measurement = {}
        for mode, measurements in config.measurements_per_generative_mode.items():
            if mode not in (DataModality.SINGLE_LABEL_CLASSIFICATION, DataModality.MULTI_LABEL_CLASSIFICATION):
                continue
            for m in measurements:
                assert m not in self.classification_mode_per_measurement
                self.classification_mode_per_measurement[m] = mode
        self._layout = None

    # ---------------------------------------------------------------------------------------------------------
    def _vocab_end(self, start):
        c = self.config
        return min(o for o in list(c.vocab_offsets_by_measurement.values()) + [c.vocab_size] if o > start)

    def _content_modules(self):
        mods = [self.ClassificationLayer, self.IsObservedLayer]
        mods += [self.regression_layers[m].proj for m in self.regression_layers]
        return mods

    def _build_layout(self):
        """Term descriptors (``esgpt_loss_term``) and column offsets of the fused head."""
        c = self.config
        V = c.vocab_size
        n_meas = len(c.measurements_idxmap)
        reg_col = {}
        col = V + n_meas
        for m in self.regression_layers:
            reg_col[m] = col
            col += self.regression_layers[m].proj.out_features
        n_content = col
        return {"V": V, "n_meas": n_meas, "reg_col": reg_col, "n_content": n_content}

    def _terms_for(self, cls_meas: set, reg_meas: set, level: int):
        c = self.config
        lay = self._layout
        terms, names = [], []
        for m, mode in self.classification_mode_per_measurement.items():
            if m not in cls_meas:
                continue
            mi = c.measurements_idxmap[m]
            vs = c.vocab_offsets_by_measurement[m]
            ve = self._vocab_end(vs)
            kind = L.TERM_SINGLE if mode == DataModality.SINGLE_LABEL_CLASSIFICATION else L.TERM_MULTI
            obs = lay["V"] + mi - 1 if kind == L.TERM_SINGLE else -1
            terms.append(L.EsgptLossTerm(kind, mi, vs, ve, vs, obs, level, 0))
            names.append(("classification", m))
        for m in c.measurements_for(DataModality.MULTIVARIATE_REGRESSION):
            if m not in reg_meas:
                continue
            mi = c.measurements_idxmap[m]
            vs = c.vocab_offsets_by_measurement[m]
            ve = vs + c.vocab_sizes_by_measurement[m]
            terms.append(L.EsgptLossTerm(L.TERM_MVREG, mi, vs, ve, lay["reg_col"][m], -1, level, 0))
            names.append(("regression", m))
        for m in c.measurements_for(DataModality.UNIVARIATE_REGRESSION):
            if m not in reg_meas:
                continue
            mi = c.measurements_idxmap[m]
            terms.append(L.EsgptLossTerm(L.TERM_UVREG, mi, 0, 0, lay["reg_col"][m], lay["V"] + mi - 1, level, 0))
            names.append(("regression", m))
        return terms, names

    def _tte_spec(self, col: int):
        c = self.config
        if c.TTE_generation_layer_type == TimeToEventGenerationHeadType.EXPONENTIAL:
            return L.EsgptTTESpec(L.TTE_EXP, 1, col, 0, 0.0, 1.0)
        return L.EsgptTTESpec(L.TTE_LNM, c.TTE_lognormal_generation_num_components, col, 0,
                              float(c.mean_log_inter_event_time_min), float(c.std_log_inter_event_time_min))

    def generation_distributions(self, encoded: torch.Tensor, cls_meas=None, reg_meas=None):
        """(classification, regression) next-event distributions of the given measurements (all when None) from
        ``encoded`` [B, L, D] (``get_classification_outputs`` / ``get_regression_outputs`` with
        ``is_generation=True``, ``model_output.py:1374-1721``): single-label (Bernoulli(is-observed),
        Categorical(vocab slice)); multi-label (None, Bernoulli(slice)); multivariate regression (None, Normal over
        all targets); univariate (Bernoulli(is-observed), Normal)."""
        c = self.config
        D_ = torch.distributions
        is_obs = self.IsObservedLayer(encoded)
        cls = {}
        todo = [(m, mode) for m, mode in self.classification_mode_per_measurement.items()
                if cls_meas is None or m in cls_meas]
        if todo:
            scores = self.ClassificationLayer(encoded)
        for m, mode in todo:
            vs = c.vocab_offsets_by_measurement[m]
            sc = scores[:, :, vs:self._vocab_end(vs)]
            if mode == DataModality.SINGLE_LABEL_CLASSIFICATION:
                cls[m] = (D_.Bernoulli(logits=is_obs[:, :, c.measurements_idxmap[m] - 1], validate_args=False),
                          D_.Categorical(logits=sc, validate_args=False))
            else:
                cls[m] = (None, D_.Bernoulli(logits=sc, validate_args=False))
        reg = {}
        for m in c.measurements_for(DataModality.MULTIVARIATE_REGRESSION):
            if reg_meas is None or m in reg_meas:
                reg[m] = (None, self.regression_layers[m](X=encoded, idx=None))
        for m in c.measurements_for(DataModality.UNIVARIATE_REGRESSION):
            if reg_meas is None or m in reg_meas:
                reg[m] = (D_.Bernoulli(logits=is_obs[:, :, c.measurements_idxmap[m] - 1], validate_args=False),
                          self.regression_layers[m](X=encoded))
        return cls, reg

    def generation_predictions(self, encoded: torch.Tensor) -> GenerativeSequenceModelPredictions:
        """Every measurement and the TTE from one encoding (the CI model, ``conditionally_independent_model.py:
        88-129`` with ``is_generation=True``)."""
        cls, reg = self.generation_distributions(encoded)
        return GenerativeSequenceModelPredictions(classification=cls, regression=reg, regression_indices={},
                                                  time_to_event=self.TTE_layer(encoded))

    def content_weight(self):
        mods = self._content_modules()
        return torch.cat([m.weight for m in mods], 0), torch.cat([m.bias for m in mods], 0)

    def _package(self, batch, losses, names):  # noqa: D401
        cls, reg = {}, {}
        for i, (kind, m) in enumerate(names):
            (cls if kind == "classification" else reg)[m] = losses[i].detach()
        loss = _TotalLoss.apply(losses)
        return GenerativeSequenceModelOutput(
            loss=loss,
            losses=GenerativeSequenceModelLosses(classification=cls, regression=reg,
                                                 time_to_event=losses[len(names)].detach()),
            preds=None,
            labels=None,
            event_mask=batch["event_mask"],
            dynamic_values_mask=batch["dynamic_values_mask"],
        )


class _TotalLoss(torch.autograd.Function):
    """``losses[-1]`` (the total of the fused losses vector) whose backward hands the incoming scalar gradient back as
    a stride-0 view over the whole vector: the fused losses' backward reads only its last element (the per-term
    entries are detached logging values), so backward needs no zero-fill + scatter launches."""

    @staticmethod
    def forward(ctx, losses):
        ctx.n = losses.shape[0]
        return losses[-1]

    @staticmethod
    def backward(ctx, g):
        return g.expand(ctx.n)


def all_classification_measurements(layer: GenerativeOutputLayerBase) -> set:
    return set(layer.classification_mode_per_measurement.keys())


def all_regression_measurements(config) -> set:
    return set(config.measurements_for(DataModality.MULTIVARIATE_REGRESSION)
               + config.measurements_for(DataModality.UNIVARIATE_REGRESSION))


def fused_ci_losses(layer: GenerativeOutputLayerBase, batch: PytorchBatch, encoded: torch.Tensor):
    """CI: one GEMM over the UNshifted encoding; the kernel reads content rows shifted by one (position 0 reads the
    head bias = Linear(zeros)), TTE rows unshifted (conditionally_independent_model.py:91-129)."""
    if layer._layout is None:
        layer._layout = layer._build_layout()
    terms, names = layer._terms_for(all_classification_measurements(layer),
                                    all_regression_measurements(layer.config), 0)
    mods = layer._content_modules() + [layer.TTE_layer.proj]
    B, Lq, D = encoded.shape
    tte = layer._tte_spec(layer._layout["n_content"])
    fused = head_losses(encoded.reshape(B * Lq, D), None, batch, terms, tte, 1, 1, mods, [])
    if fused is not None:
        return fused, names
    z = linear_bias(encoded.reshape(B * Lq, D), [m.weight for m in mods], [m.bias for m in mods])
    b = torch.cat([m.bias for m in mods], 0)
    losses = output_loss(z, None, b, batch, terms, tte, 1, 1)
    return losses, names


def fused_na_losses(layer: GenerativeOutputLayerBase, batch: PytorchBatch, encoded: torch.Tensor):
    """NA: level i (1..G-1) measurements are predicted from encoded[:, :, i-1] (no shift); TTE from the last level
    (nested_attention_model.py:115-197)."""
    if layer._layout is None:
        layer._layout = layer._build_layout()
    c = layer.config
    B, Lq, G, D = encoded.shape
    cls_all = all_classification_measurements(layer)
    reg_all = all_regression_measurements(c)
    terms, names = [], []
    seen = set()
    for i in range(1, G):
        cat, num = _level_sets(c.measurements_per_dep_graph_level[i])
        t, n = layer._terms_for(cat & cls_all, num & reg_all, i - 1)
        for tt, nn_ in zip(t, n):
            if nn_ in seen:  # the reference's dict.update keeps the last level's value
                idx = names.index(nn_)
                terms.pop(idx)
                names.pop(idx)
            seen.add(nn_)
            terms.append(tt)
            names.append(nn_)
    mods = layer._content_modules()
    if terms:
        from ..fused import GEMM_DTYPES, compute_dtype
        from .structured_attention import split_last_level

        dt = compute_dtype()
        if encoded.is_cuda and dt in GEMM_DTYPES and G >= 2 and D % 8 == 0:
            # the content levels and the TTE level as the head GEMM's operands, split and cast in one pass (one
            # pass back in the backward)
            from ..kernels import _ops

            head, last = _ops().na_head_split(encoded, dt)
        else:
            head, last = split_last_level(encoded)  # one cat in backward instead of two zero-filled slice gradients
        fused = head_losses(head.reshape(B * Lq * (G - 1), D), last.reshape(B * Lq, D), batch, terms,
                            layer._tte_spec(0), 0, max(1, G - 1), mods, [layer.TTE_layer.proj])
        if fused is not None:
            return fused, names
    if terms:
        zc = linear_bias(encoded[:, :, : G - 1, :].reshape(B * Lq * (G - 1), D), [m.weight for m in mods],
                         [m.bias for m in mods])
    else:
        zc = torch.zeros(1, 1, device=encoded.device, dtype=encoded.dtype)
    zt = linear_bias(encoded[:, :, G - 1, :].reshape(B * Lq, D), [layer.TTE_layer.proj.weight],
                     [layer.TTE_layer.proj.bias])
    losses = output_loss(zc, zt, None, batch, terms, layer._tte_spec(0), 0, max(1, G - 1))
    return losses, names
