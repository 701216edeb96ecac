"""Output containers and the fused generative output layer (``EventStream/transformer/model_output.py``).

``GenerativeOutputLayerBase`` keeps the reference's submodules and parameter names (``TTE_layer``,
``IsObservedLayer``, ``ClassificationLayer``, ``regression_layers``; ``:1253-1309``). Training losses follow
``get_TTE_outputs`` / ``get_classification_outputs`` / ``get_regression_outputs`` (``:1311-1721``) but are
computed by ONE head GEMM (all heads' weights concatenated along the output dimension) plus the fused loss kernel
(``kernels.OutputLossFn``), which also produces d(loss)/d(logits).

Head column layout of the fused GEMM: [ClassificationLayer (V) | IsObservedLayer (n_meas) |
regression_layers[m].proj (in measurements_per_generative_mode order) || TTE_layer.proj].
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from transformers.utils import ModelOutput

from .. import _lib as L
from ..data.data_embedding_enums import MeasIndexGroupOptions
from ..data.types import DataModality, PytorchBatch
from ..fused import head_losses, linear_bias
from ..kernels import OutputLossFn, batch_view
from .config import TimeToEventGenerationHeadType
from .generative_layers import (
    ExponentialTTELayer,
    GaussianIndexedRegressionLayer,
    GaussianRegressionLayer,
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


@dataclass
class GenerativeSequenceModelPredictions(ModelOutput):
    classification: dict | None = None
    regression: dict | None = None
    regression_indices: dict | None = None
    time_to_event: torch.distributions.Distribution | None = None


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

    def content_weight(self):
        mods = self._content_modules()
        return torch.cat([m.weight for m in mods], 0), torch.cat([m.bias for m in mods], 0)

    def _package(self, batch, losses, names):
        cls, reg = {}, {}
        for i, (kind, m) in enumerate(names):
            (cls if kind == "classification" else reg)[m] = losses[i].detach()
        loss = losses[-1]
        return GenerativeSequenceModelOutput(
            loss=loss,
            losses=GenerativeSequenceModelLosses(classification=cls, regression=reg,
                                                 time_to_event=losses[len(names)].detach()),
            preds=None,
            labels=None,
            event_mask=batch["event_mask"],
            dynamic_values_mask=batch["dynamic_values_mask"],
        )


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
    bv = batch_view(batch)
    tte = layer._tte_spec(layer._layout["n_content"])
    fused = head_losses(encoded.reshape(B * Lq, D), None, bv, terms, tte, 1, 1, mods, [])
    if fused is not None:
        return fused, names
    z = linear_bias(encoded.reshape(B * Lq, D), [m.weight for m in mods], [m.bias for m in mods])
    b = torch.cat([m.bias for m in mods], 0)
    losses = OutputLossFn.apply(z, None, b, bv, terms, tte, 1, 1)
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
    bv = batch_view(batch)
    if terms:
        fused = head_losses(encoded[:, :, : G - 1, :].reshape(B * Lq * (G - 1), D),
                            encoded[:, :, G - 1, :].reshape(B * Lq, D), bv, terms, layer._tte_spec(0), 0,
                            max(1, G - 1), mods, [layer.TTE_layer.proj])
        if fused is not None:
            return fused, names
    if terms:
        zc = linear_bias(encoded[:, :, : G - 1, :].reshape(B * Lq * (G - 1), D), [m.weight for m in mods],
                         [m.bias for m in mods])
    else:
        zc = torch.zeros(1, 1, device=encoded.device, dtype=encoded.dtype)
    zt = linear_bias(encoded[:, :, G - 1, :].reshape(B * Lq, D), [layer.TTE_layer.proj.weight],
                     [layer.TTE_layer.proj.bias])
    losses = OutputLossFn.apply(zc, zt, None, bv, terms, layer._tte_spec(0), 0, max(1, G - 1))
    return losses, names
