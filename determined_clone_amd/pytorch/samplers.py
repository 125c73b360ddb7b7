"""Samplers that make data loading resumable and rank-sharded
(reference: `harness/determined/pytorch/samplers.py`)."""
from typing import Iterator

import numpy as np
import torch


class RepeatSampler(torch.utils.data.Sampler):
    """Infinitely repeat a sampler (epochs are tracked by the controller, not the iterator)."""

    def __init__(self, sampler) -> None:
        self._sampler = sampler

    def __len__(self) -> int:
        return len(self._sampler)

    def __iter__(self) -> Iterator:
        while True:
            yield from self._sampler


class RepeatBatchSampler(torch.utils.data.BatchSampler):
    def __init__(self, batch_sampler) -> None:
        self._batch_sampler = batch_sampler

    def __len__(self) -> int:
        return len(self._batch_sampler)

    def __iter__(self) -> Iterator:
        while True:
            yield from self._batch_sampler


class DistributedSampler(torch.utils.data.Sampler):
    """Every ``num_workers``-th record starting at ``rank`` (no padding; last partial dropped
    consistently across ranks)."""

    def __init__(self, sampler, num_workers: int, rank: int) -> None:
        self._sampler = sampler
        self._num_workers = num_workers
        self._rank = rank

    def __len__(self) -> int:
        n = len(self._sampler)
        return n // self._num_workers + (1 if self._rank < n % self._num_workers else 0)

    def __iter__(self) -> Iterator:
        for i, x in enumerate(self._sampler):
            if i % self._num_workers == self._rank:
                yield x


class DistributedBatchSampler(torch.utils.data.BatchSampler):
    """Shard a batch sampler across ``num_workers`` ranks by dealing whole batches round-robin:
    rank r yields batches r, r + num_workers, r + 2 * num_workers, ... of the wrapped sampler (each
    unchanged). Built on a per-slot batch sampler, the ``num_workers`` consecutive per-slot batches
    that one step consumes together form that step's global batch."""

    def __init__(self, batch_sampler, num_workers: int, rank: int) -> None:
        self._batch_sampler = batch_sampler
        self._num_workers = num_workers
        self._rank = rank

    def __len__(self) -> int:
        n = len(self._batch_sampler)
        return n // self._num_workers + (1 if self._rank < n % self._num_workers else 0)

    def __iter__(self) -> Iterator:
        for i, b in enumerate(self._batch_sampler):
            if i % self._num_workers == self._rank:
                yield b


class SkipSampler(torch.utils.data.Sampler):
    def __init__(self, sampler, skip: int) -> None:
        self._sampler = sampler
        self._skip = skip

    def __len__(self) -> int:
        return len(self._sampler)

    def __iter__(self) -> Iterator:
        it = iter(self._sampler)
        for _ in range(self._skip):
            next(it)
        yield from it


class SkipBatchSampler(torch.utils.data.BatchSampler):
    def __init__(self, batch_sampler, skip: int) -> None:
        self._batch_sampler = batch_sampler
        self._skip = skip

    def __len__(self) -> int:
        return len(self._batch_sampler)

    def __iter__(self) -> Iterator:
        it = iter(self._batch_sampler)
        for _ in range(self._skip):
            next(it)
        yield from it


class ReproducibleShuffleSampler(torch.utils.data.Sampler):
    """Shuffle with a per-epoch seed derived from ``seed`` so a restarted trial replays the same
    order."""

    def __init__(self, sampler, seed: int) -> None:
        self._sampler = sampler
        self._seed = seed
        self._epoch = 0

    def __iter__(self) -> Iterator:
        items = list(self._sampler)
        rng = np.random.RandomState(self._seed + self._epoch)
        self._epoch += 1
        rng.shuffle(items)
        return iter(items)

    def __len__(self) -> int:
        return len(self._sampler)


class ReproducibleShuffleBatchSampler(torch.utils.data.Sampler):
    def __init__(self, batch_sampler, seed: int) -> None:
        self._batch_sampler = batch_sampler
        self._seed = seed
        self._epoch = 0

    def __iter__(self) -> Iterator:
        batches = list(self._batch_sampler)
        rng = np.random.RandomState(self._seed + self._epoch)
        self._epoch += 1
        rng.shuffle(batches)
        return iter(batches)

    def __len__(self) -> int:
        return len(self._batch_sampler)
