import random

import numpy as np
import torch


def seed_everything(seed=0, *a, **k):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    return seed


class LightningModule(torch.nn.Module):
    pass
