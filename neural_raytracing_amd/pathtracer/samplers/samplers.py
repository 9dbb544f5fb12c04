import torch
import torch.nn as nn


class Sampler(nn.Module):
    """Independent sampler (samplers.py:4-26): ``sample(shape) = torch.rand(shape)``."""

    def __init__(self, sample_count=0, device="cuda"):
        super().__init__()
        self.sample_count = sample_count
        self.device = device

    def sample(self, shape, device=None):
        if device is None:
            device = self.device
        return torch.rand(shape, device=device)
