"""Distribution heads — drop-in for ``EventStream/transformer/generative_layers.py:1-184``.

Parameter layout is unchanged (``proj`` Linear in every head). In training, the heads' projections are fused
into the output layer's single head GEMM and their log-likelihoods are evaluated inside the fused loss kernel
(``csrc/losses.hip``); ``forward`` still returns the reference's distribution objects (for metrics / sampling),
built with ``validate_args=False``: torch's argument validation is a device->host read per distribution, which
dominated the per-event cost of generation.
"""
from __future__ import annotations

import torch
from torch import distributions as D


class LogNormalMixtureDistribution(D.TransformedDistribution):
    """Mixture of LogNormals = Exp(affine(Gaussian mixture)); restates the third-party
    ``pytorch_lognormal_mixture.LogNormalMixtureDistribution`` (0.0.1) API used by the reference."""

    def __init__(self, locs, log_scales, log_weights, mean_log_inter_time: float = 0.0,
                 std_log_inter_time: float = 1.0, validate_args=False):
        gmm = D.MixtureSameFamily(D.Categorical(logits=log_weights, validate_args=False),
                                 D.Normal(loc=locs, scale=log_scales.exp(), validate_args=False), validate_args=False)
        transforms = []
        if not (mean_log_inter_time == 0.0 and std_log_inter_time == 1.0):
            transforms.append(D.AffineTransform(loc=mean_log_inter_time, scale=std_log_inter_time))
        transforms.append(D.ExpTransform())
        self.mean_log_inter_time = mean_log_inter_time
        self.std_log_inter_time = std_log_inter_time
        self.params = (locs, log_scales, log_weights)
        super().__init__(gmm, transforms, validate_args=validate_args)

    @property
    def mean(self):
        a, b = self.std_log_inter_time, self.mean_log_inter_time
        comp = self.base_dist.component_distribution
        logits = self.base_dist.mixture_distribution.logits
        return (logits + a * comp.loc + b + 0.5 * a**2 * comp.variance).logsumexp(-1).exp()


class LogNormalMixtureTTELayer(torch.nn.Module):
    def __init__(self, in_dim: int, num_components: int, mean_log_inter_time: float = 0.0,
                 std_log_inter_time: float = 1.0):
        super().__init__()
        self.proj = torch.nn.Linear(in_dim, 3 * num_components)
        self.num_components = num_components
        self.mean_log_inter_time = mean_log_inter_time
        self.std_log_inter_time = std_log_inter_time

    def forward(self, T: torch.Tensor) -> LogNormalMixtureDistribution:
        p = self.proj(T)
        return LogNormalMixtureDistribution(p[..., 0::3], p[..., 1::3], p[..., 2::3], self.mean_log_inter_time,
                                            self.std_log_inter_time)


class ExponentialTTELayer(torch.nn.Module):
    def __init__(self, in_dim: int):
        super().__init__()
        self.proj = torch.nn.Linear(in_dim, 1)

    def forward(self, T: torch.Tensor) -> D.Exponential:
        rate = torch.nn.functional.elu(self.proj(T)) + 1 + torch.finfo(T.dtype).tiny
        return D.Exponential(rate=rate.squeeze(dim=-1), validate_args=False)


class GaussianIndexedRegressionLayer(torch.nn.Module):
    def __init__(self, n_regression_targets: int, in_dim: int):
        super().__init__()
        self.proj = torch.nn.Linear(in_dim, n_regression_targets * 2)

    def forward(self, X: torch.Tensor, idx: torch.LongTensor | None = None) -> D.Normal:
        Z = self.proj(X)
        mean = Z[..., 0::2]
        std = torch.nn.functional.elu(Z[..., 1::2]) + 1 + torch.finfo(X.dtype).tiny
        if idx is None:
            return D.Normal(loc=mean, scale=std, validate_args=False)
        return D.Normal(loc=mean.gather(-1, idx), scale=std.gather(-1, idx), validate_args=False)


class GaussianRegressionLayer(torch.nn.Module):
    def __init__(self, in_dim: int):
        super().__init__()
        self.proj = torch.nn.Linear(in_dim, 2)

    def forward(self, X: torch.Tensor) -> D.Normal:
        Z = self.proj(X)
        std = torch.nn.functional.elu(Z[..., 1::2]) + 1 + torch.finfo(X.dtype).tiny
        return D.Normal(loc=Z[..., 0::2], scale=std, validate_args=False)
