"""MNIST CNN of the reference tutorial (reference: `examples/tutorials/mnist_pytorch/model.py`:
conv32-conv64-maxpool-dropout-fc128-dropout-fc10, log-softmax output) + an offline dataset.

No network here: :func:`get_dataset` reads the standard IDX files from ``data_dir`` if present and
otherwise generates a deterministic synthetic MNIST-shaped dataset (class-dependent blobs, so the
task is learnable and validation accuracy is meaningful in tests)."""
import gzip
import os
import pathlib
from typing import Any, Dict, Optional

import numpy as np
import torch
from torch import nn


class Flatten(nn.Module):
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x.reshape(x.shape[0], -1)


def build_model(hparams: Dict[str, Any]) -> nn.Module:
    return nn.Sequential(
        nn.Conv2d(1, int(hparams["n_filters1"]), 3, 1),
        nn.ReLU(),
        nn.Conv2d(int(hparams["n_filters1"]), int(hparams["n_filters2"]), 3),
        nn.ReLU(),
        nn.MaxPool2d(2),
        nn.Dropout2d(float(hparams["dropout1"])),
        Flatten(),
        nn.Linear(144 * int(hparams["n_filters2"]), 128),
        nn.ReLU(),
        nn.Dropout(float(hparams["dropout2"])),
        nn.Linear(128, 10),
        nn.LogSoftmax(dim=1),
    )


def _read_idx(path: pathlib.Path) -> np.ndarray:
    opener = gzip.open if path.suffix == ".gz" else open
    with opener(path, "rb") as f:
        data = f.read()
    ndim = data[3]
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


class SyntheticMNIST(torch.utils.data.Dataset):
    """Deterministic 28x28 digit-like data: each class is a distinct blob pattern + noise."""

    def __init__(self, n: int, seed: int) -> None:
        g = np.random.RandomState(seed)
        proto = np.random.RandomState(1234).rand(10, 28, 28).astype(np.float32)
        proto = (proto > 0.7).astype(np.float32)
        self.y = g.randint(0, 10, size=n).astype(np.int64)
        self.x = (proto[self.y] + 0.3 * g.randn(n, 28, 28).astype(np.float32))[:, None]
        self.x = (self.x - 0.1307) / 0.3081

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, i: int):
        return torch.from_numpy(self.x[i]), int(self.y[i])


class IDXMNIST(torch.utils.data.Dataset):
    def __init__(self, images: np.ndarray, labels: np.ndarray) -> None:
        self.x = ((images.astype(np.float32) / 255.0 - 0.1307) / 0.3081)[:, None]
        self.y = labels.astype(np.int64)

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, i: int):
        return torch.from_numpy(self.x[i]), int(self.y[i])


def get_dataset(data_dir: Optional[os.PathLike], train: bool, synthetic_size: Optional[int] = None):
    prefix = "train" if train else "t10k"
    if data_dir is not None:
        d = pathlib.Path(data_dir)
        for suffix in ("", ".gz"):
            img = d / f"{prefix}-images-idx3-ubyte{suffix}"
            lab = d / f"{prefix}-labels-idx1-ubyte{suffix}"
            if img.exists() and lab.exists():
                return IDXMNIST(_read_idx(img), _read_idx(lab))
    n = synthetic_size or (60000 if train else 10000)
    return SyntheticMNIST(n, seed=0 if train else 1)
