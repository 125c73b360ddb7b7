"""Shared pieces of the two batch-inference implementations: a CIFAR-10-shaped synthetic dataset
(no download in this environment) and a small random-init convnet in NHWC."""
import torch
from torch import nn


class SyntheticCifar(torch.utils.data.Dataset):
    def __init__(self, n: int = 512, seed: int = 0) -> None:
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, 3, 32, 32, generator=g)

    def __len__(self) -> int:
        return len(self.x)

    def __getitem__(self, i: int):
        return i, self.x[i]


def build_model() -> nn.Module:
    torch.manual_seed(0)
    return nn.Sequential(
        nn.Conv2d(3, 32, 3, padding=1), nn.ReLU(), nn.MaxPool2d(2),
        nn.Conv2d(32, 64, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(1),
        nn.Flatten(), nn.Linear(64, 10))
