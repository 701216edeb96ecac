"""Restatement of the third-party `pytorch-lognormal-mixture==0.0.1` (pinned at the reference's
env.yml:409; not installable here). Published algorithm: a LogNormal mixture is the ExpTransform of a
Gaussian mixture, optionally preceded by the affine map y -> mean_log + std_log * y when
(mean_log, std_log) != (0, 1). Pinned by the reference's known answers at (0, 1)
(tests/transformer/test_generative_layers.py, test_model_output.py LL -7.6554941334115565).
Used ONLY to run the reference for golden vectors."""
import torch
from torch import distributions as D


class LogNormalMixtureDistribution(D.TransformedDistribution):
    def __init__(self, locs, log_scales, log_weights, mean_log_inter_time=0.0, std_log_inter_time=1.0,
                 validate_args=None):
        mixture_dist = D.Categorical(logits=log_weights)
        component_dist = D.Normal(loc=locs, scale=log_scales.exp())
        GMM = D.MixtureSameFamily(mixture_dist, component_dist)
        if mean_log_inter_time == 0.0 and std_log_inter_time == 1.0:
            transforms = []
        else:
            transforms = [D.AffineTransform(loc=mean_log_inter_time, scale=std_log_inter_time)]
        self.mean_log_inter_time = mean_log_inter_time
        self.std_log_inter_time = std_log_inter_time
        transforms.append(D.ExpTransform())
        self.transforms = transforms
        super().__init__(GMM, transforms, validate_args=validate_args)

    @property
    def mean(self):
        a = self.std_log_inter_time
        b = self.mean_log_inter_time
        loc = self.base_dist._component_distribution.loc
        variance = self.base_dist._component_distribution.variance
        log_weights = self.base_dist._mixture_distribution.logits
        return (log_weights + a * loc + b + 0.5 * a**2 * variance).logsumexp(-1).exp()
