"""Determined-style DataLoader + batch helpers (reference: `harness/determined/pytorch/_data.py`).

The wrapper records the user's dataset/sampler configuration and builds the real
``torch.utils.data.DataLoader`` only in :meth:`DataLoader.get_data_loader`, where the controller
injects repeat (training), rank sharding and skip (resume mid-epoch) into the batch sampler so a
restarted trial continues at exactly the next batch.

MI355X additions: :class:`DevicePrefetcher` overlaps the host->device copy of batch ``i+1`` with
step ``i`` on a side HIP stream (pinned memory, ``non_blocking``), and :class:`SyntheticDataset`
keeps a fixed batch resident on the GPU for throughput benchmarks.
"""
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import torch
from torch.utils.data import BatchSampler, Dataset, RandomSampler, SequentialSampler
from torch.utils.data import _utils

from determined_clone_amd.pytorch import samplers

TorchData = Union[Dict[str, torch.Tensor], Sequence[torch.Tensor], torch.Tensor]


class DataLoader:
    def __init__(self, dataset: Dataset, batch_size: Optional[int] = 1, shuffle: bool = False,
                 sampler: Any = None, batch_sampler: Any = None, num_workers: int = 0,
                 collate_fn: Optional[Callable] = None, pin_memory: bool = False,
                 drop_last: bool = False, timeout: float = 0,
                 worker_init_fn: Optional[Callable] = None, multiprocessing_context: Any = None,
                 generator: Any = None, *, prefetch_factor: Optional[int] = None,
                 persistent_workers: bool = False) -> None:
        if isinstance(dataset, torch.utils.data.IterableDataset):
            raise ValueError("IterableDatasets are not supported by DataLoader(); shard/repeat/skip "
                             "them yourself and return a torch DataLoader from the trial instead")
        # batch_size=None (no auto-collation: every item is already a batch) is supported here,
        # unlike the reference; the sampler chain then shards/repeats/skips whole batches.
        if num_workers < 0:
            raise ValueError("num_workers option should be non-negative")
        if timeout < 0:
            raise ValueError("timeout option should be non-negative")
        if num_workers == 0 and prefetch_factor is not None:
            raise ValueError("prefetch_factor needs num_workers > 0")
        if num_workers > 0 and prefetch_factor is None:
            prefetch_factor = 2
        if persistent_workers and num_workers == 0:
            raise ValueError("persistent_workers option needs num_workers > 0")
        if sampler is not None and shuffle:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        if batch_sampler is not None:
            if batch_size != 1 or shuffle or sampler is not None or drop_last:
                raise ValueError("batch_sampler option is mutually exclusive with batch_size, "
                                 "shuffle, sampler, and drop_last")
            batch_size = None
            drop_last = False
        elif batch_size is None and (shuffle or drop_last):
            raise ValueError("batch_size=None is mutually exclusive with shuffle and drop_last")
        if sampler is None:
            sampler = RandomSampler(dataset, generator=generator) if shuffle else SequentialSampler(dataset)
        if batch_size is not None and batch_sampler is None:
            batch_sampler = BatchSampler(sampler, batch_size, drop_last)
        self.dataset = dataset
        self.num_workers = num_workers
        self.prefetch_factor = prefetch_factor
        self.pin_memory = pin_memory
        self.timeout = timeout
        self.worker_init_fn = worker_init_fn
        self.multiprocessing_context = multiprocessing_context
        self.batch_size = batch_size
        self.drop_last = drop_last
        self.sampler = sampler
        self.batch_sampler = batch_sampler
        self.generator = generator
        self.persistent_workers = persistent_workers
        if collate_fn is None:
            collate_fn = _utils.collate.default_collate if batch_sampler is not None else _utils.collate.default_convert
        self.collate_fn = collate_fn

    def get_data_loader(self, repeat: bool = False, skip: int = 0, num_replicas: int = 1,
                        rank: int = 0) -> torch.utils.data.DataLoader:
        if self.batch_sampler is None:
            # batch_size=None: every dataset item already is a batch.
            s = self.sampler
            if repeat:
                s = samplers.RepeatSampler(s)
            if num_replicas > 1:
                s = samplers.DistributedSampler(s, num_replicas, rank)
            if skip > 0:
                s = samplers.SkipSampler(s, skip)
            return torch.utils.data.DataLoader(
                self.dataset, batch_size=None, sampler=s, num_workers=self.num_workers,
                collate_fn=self.collate_fn, pin_memory=self.pin_memory, timeout=self.timeout,
                worker_init_fn=self.worker_init_fn, generator=self.generator,
                prefetch_factor=self.prefetch_factor, persistent_workers=self.persistent_workers)
        bs = adapt_batch_sampler(self.batch_sampler, repeat=repeat, skip=skip,
                                 num_replicas=num_replicas, rank=rank)
        return torch.utils.data.DataLoader(
            self.dataset, batch_sampler=bs, num_workers=self.num_workers,
            collate_fn=self.collate_fn, pin_memory=self.pin_memory, timeout=self.timeout,
            worker_init_fn=self.worker_init_fn, multiprocessing_context=self.multiprocessing_context,
            generator=self.generator, prefetch_factor=self.prefetch_factor,
            persistent_workers=self.persistent_workers)

    def __iter__(self) -> Iterator:
        return iter(self.get_data_loader())

    def __len__(self) -> int:
        return len(self.batch_sampler if self.batch_sampler is not None else self.sampler)


def adapt_batch_sampler(batch_sampler: BatchSampler, repeat: bool = False, skip: int = 0,
                        num_replicas: int = 1, rank: int = 0) -> BatchSampler:
    """repeat -> shard -> skip (skip counts per-rank batches already consumed)."""
    if repeat:
        batch_sampler = samplers.RepeatBatchSampler(batch_sampler)
    if num_replicas > 1:
        batch_sampler = samplers.DistributedBatchSampler(batch_sampler, num_replicas, rank)
    if skip > 0:
        batch_sampler = samplers.SkipBatchSampler(batch_sampler, skip)
    return batch_sampler


def data_length(data: TorchData) -> int:
    if isinstance(data, torch.Tensor):
        return len(data)
    if isinstance(data, dict):
        vals = list(data.values())
        return data_length(vals[0]) if vals else 0
    if isinstance(data, (list, tuple)):
        return data_length(data[0]) if data else 0
    raise TypeError(f"cannot infer batch length of {type(data).__name__}")


def to_device(data: Any, device: torch.device, warned_types: Optional[set] = None,
              non_blocking: bool = True) -> Any:
    if isinstance(data, torch.Tensor):
        return data.to(device, non_blocking=non_blocking and data.is_pinned() if data.device.type == "cpu" else non_blocking)
    if isinstance(data, dict):
        return {k: to_device(v, device, warned_types, non_blocking) for k, v in data.items()}
    if isinstance(data, tuple) and hasattr(data, "_fields"):
        return type(data)(*(to_device(v, device, warned_types, non_blocking) for v in data))
    if isinstance(data, (list, tuple)):
        return type(data)(to_device(v, device, warned_types, non_blocking) for v in data)
    if hasattr(data, "to") and callable(data.to):
        return data.to(device)
    return data


class DevicePrefetcher:
    """Wrap a batch iterator: copies batch i+1 to the GPU on a side stream while step i runs."""

    def __init__(self, it: Iterator, device: torch.device) -> None:
        self._it = it
        self._device = device
        self._stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self._next: Any = None
        self._done = False
        self._preload()

    def _preload(self) -> None:
        try:
            batch = next(self._it)
        except StopIteration:
            self._done = True
            self._next = None
            return
        if self._stream is None:
            self._next = to_device(batch, self._device)
            return
        with torch.cuda.stream(self._stream):
            self._next = to_device(batch, self._device)

    def __iter__(self) -> "DevicePrefetcher":
        return self

    def __next__(self) -> Any:
        if self._done and self._next is None:
            raise StopIteration
        if self._stream is not None:
            torch.cuda.current_stream(self._device).wait_stream(self._stream)
            _record_stream(self._next, torch.cuda.current_stream(self._device))
        out = self._next
        self._preload()
        return out


def _record_stream(data: Any, stream: Any) -> None:
    if isinstance(data, torch.Tensor):
        if data.is_cuda:
            data.record_stream(stream)
    elif isinstance(data, dict):
        for v in data.values():
            _record_stream(v, stream)
    elif isinstance(data, (list, tuple)):
        for v in data:
            _record_stream(v, stream)


class SyntheticDataset(Dataset):
    """A fixed pool of random samples (benchmarks: "data": "synthetic"). ``length`` is the
    virtual epoch size; items cycle through ``pool`` pre-generated samples."""

    def __init__(self, length: int, make_sample: Callable[[int], Any], pool: int = 64) -> None:
        self.length = length
        self.samples = [make_sample(i) for i in range(pool)]

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> Any:
        return self.samples[i % len(self.samples)]


class DeviceBatchDataset(Dataset):
    """Whole pre-collated batches already resident in HBM; item i is batch i % n. Used with
    ``batch_size=None`` so the loader does no collation or copies (synthetic benchmarking)."""

    def __init__(self, batches: List[Any], length: int) -> None:
        self.batches = batches
        self.length = length

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int) -> Any:
        return self.batches[i % len(self.batches)]
