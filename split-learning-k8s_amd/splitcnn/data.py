"""Synthetic MNIST-shape batches.

The reference trains on torchvision MNIST normalised with (0.1307, 0.3081) (src/client_part.py:61-64,
98); there is no network here, so batches are class prototypes plus noise pushed through the same
normalisation. Generated on the CPU from a seeded torch.Generator so every machine with this torch
build produces bit-identical batches (the golden loss curve depends on it).
"""
from __future__ import annotations

import torch

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081


class SyntheticMNIST:
    def __init__(self, seed: int = 42):
        self.gen = torch.Generator().manual_seed(seed)
        self.proto = torch.rand(10, 1, 28, 28, generator=self.gen)

    def batch(self, B: int):
        y = torch.randint(0, 10, (B,), generator=self.gen)
        x = (self.proto[y] + 0.3 * torch.randn(B, 1, 28, 28, generator=self.gen) - MNIST_MEAN) / MNIST_STD
        return x.contiguous(), y


def init_models(seed: int = 0, full: bool = False):
    """Seeded default init in the reference order (conv1, then conv2, fc1)."""
    from .model_def import FullModel, ModelPartA, ModelPartB
    torch.manual_seed(seed)
    if full:
        return FullModel()
    a = ModelPartA()
    b = ModelPartB()
    return a, b
