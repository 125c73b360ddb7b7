"""CIFAR-10 CNN used for the adaptive_asha search config (reference: the CIFAR-10 PyTorch example
of the e2e fixtures / docs: 4 conv layers + dropout + 2 FC). NHWC bf16-friendly: the conv stack runs
channels_last, BatchNorm+ReLU uses the fused HIP kernel on the GPU. Offline synthetic data."""
import fcntl
import os
import tempfile
from typing import Any, Dict, Optional

import numpy as np
import torch
from torch import nn

from determined_clone_amd.models.resnet import BatchNormAct2d


class CifarCNN(nn.Module):
    def __init__(self, hparams: Dict[str, Any]) -> None:
        super().__init__()
        w = int(hparams.get("width", 32))
        d = float(hparams.get("dropout", 0.25))
        self.features = nn.Sequential(
            nn.Conv2d(3, w, 3, padding=1, bias=False), BatchNormAct2d(w),
            nn.Conv2d(w, w, 3, padding=1, bias=False), BatchNormAct2d(w),
            nn.MaxPool2d(2), nn.Dropout(d),
            nn.Conv2d(w, 2 * w, 3, padding=1, bias=False), BatchNormAct2d(2 * w),
            nn.Conv2d(2 * w, 2 * w, 3, padding=1, bias=False), BatchNormAct2d(2 * w),
            nn.MaxPool2d(2), nn.Dropout(d),
        )
        self.head = nn.Sequential(nn.Flatten(), nn.Linear(2 * w * 8 * 8, int(hparams.get("hidden", 512))),
                                  nn.ReLU(), nn.Dropout(float(hparams.get("dropout2", 0.5))),
                                  nn.Linear(int(hparams.get("hidden", 512)), 10))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.head(self.features(x))


class SyntheticCIFAR10(torch.utils.data.Dataset):
    """Deterministic 32x32x3 class-conditional data: learnable, but not at a glance.

    Each image is ``signal`` x a smooth class prototype, cropped at a random offset of up to
    ``max_shift`` pixels (so position varies), plus unit Gaussian noise; ``label_noise`` of the
    training labels are replaced by random classes. A small CNN needs several epochs and a sane
    learning rate to get the validation error down (too high a rate diverges), so an HP search
    sees a real spread of validation errors -- what ASHA's promotions act on. Stored as fp16
    (50,000 records: 307 MB, one shared copy per node -- see ``cache_dir``)."""

    def __init__(self, n: int, seed: int, signal: float = 0.12, label_noise: float = 0.1,
                 max_shift: int = 4, cache_dir: Optional[str] = None) -> None:
        """``cache_dir`` (default ``$DET_DATA_CACHE`` or the temp dir): the arrays are generated
        once per parameter set into ``<cache_dir>/dca_synthetic_cifar/`` (under a file lock) and
        memory-mapped by every later instance -- the 16 trial processes of an HP search share one
        page-cache copy instead of each spending seconds generating 307 MB at start-up."""
        cache_dir = cache_dir or os.environ.get("DET_DATA_CACHE") or tempfile.gettempdir()
        key = f"n{n}_s{seed}_sig{signal}_ln{label_noise}_sh{max_shift}_v1"
        d = os.path.join(cache_dir, "dca_synthetic_cifar")
        try:
            os.makedirs(d, exist_ok=True)
            xp, yp = os.path.join(d, key + ".x.npy"), os.path.join(d, key + ".y.npy")
            with open(os.path.join(d, key + ".lock"), "w") as lk:
                fcntl.flock(lk, fcntl.LOCK_EX)
                if not (os.path.exists(xp) and os.path.exists(yp)):
                    self._generate(n, seed, signal, label_noise, max_shift)
                    for path, arr in ((xp, self.x), (yp, self.y)):
                        tmp = f"{path}.{os.getpid()}.tmp.npy"
                        np.save(tmp, arr)
                        os.replace(tmp, path)
            self.x = np.load(xp, mmap_mode="r")
            self.y = np.load(yp)
        except OSError:  # read-only / full cache dir: generate in memory
            self._generate(n, seed, signal, label_noise, max_shift)

    def _generate(self, n: int, seed: int, signal: float, label_noise: float, max_shift: int) -> None:
        g = np.random.RandomState(seed)
        side = 32 + 2 * max_shift
        proto = torch.from_numpy(np.random.RandomState(99).randn(10, 3, side, side).astype(np.float32))
        proto = torch.nn.functional.avg_pool2d(proto, 5, 1, 2)
        proto = (proto / proto.std()).numpy()
        y_true = g.randint(0, 10, size=n)
        dx = g.randint(0, 2 * max_shift + 1, size=n)
        dy = g.randint(0, 2 * max_shift + 1, size=n)
        x = g.randn(n, 3, 32, 32).astype(np.float32)
        for i in range(n):
            x[i] += signal * proto[y_true[i], :, dy[i]:dy[i] + 32, dx[i]:dx[i] + 32]
        self.x = x.astype(np.float16)
        flip = g.rand(n) < label_noise
        self.y = np.where(flip, g.randint(0, 10, size=n), y_true).astype(np.int64)

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, i: int):
        # fp16 as stored (exact): the consumer converts on its device (examples/cifar10_asha)
        return torch.from_numpy(np.ascontiguousarray(self.x[i])), int(self.y[i])

    def __getitems__(self, idx):
        """Batched fetch (torch's DataLoader calls this with a batch's indices): one vectorised
        memmap gather, returned already collated as a :class:`CifarBatch` (pass
        ``collate_fn=collate``). Fetching record by record, converting to fp32 on the CPU and
        stacking cost ~3 ms of CPU per 128-record batch -- paid by each of the 16 trial processes
        of an ASHA search sharing the node's cores. Images stay fp16 (exact): no CPU conversion,
        which in torch would also fan out over every intra-op thread of every trial process."""
        idx = np.asarray(idx, dtype=np.int64)
        return CifarBatch(torch.from_numpy(self.x[idx]), torch.from_numpy(self.y[idx]))


class CifarBatch(tuple):
    """(images [B, 3, 32, 32] fp16, labels [B] int64) of :meth:`SyntheticCIFAR10.__getitems__`."""

    def __new__(cls, x: torch.Tensor, y: torch.Tensor) -> "CifarBatch":
        return super().__new__(cls, (x, y))


def collate(batch):
    """DataLoader ``collate_fn`` for :class:`SyntheticCIFAR10`: a batched fetch is already a batch;
    anything else (a list of records) goes through torch's default collation."""
    if isinstance(batch, CifarBatch):
        return tuple(batch)
    return torch.utils.data.default_collate(batch)
