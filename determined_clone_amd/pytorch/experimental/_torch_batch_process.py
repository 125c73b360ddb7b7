"""Distributed batch inference / processing over a dataset (reference:
`harness/determined/pytorch/experimental/_torch_batch_process.py`).

``torch_batch_process(MyProcessor, dataset, batch_size=..., checkpoint_interval=...)`` shards the
dataset across all workers (one per MI355X), calls ``MyProcessor.process_batch`` on each shard's
batches, and every ``checkpoint_interval`` batches synchronises the workers, records
``steps_completed`` in a checkpoint (so a preempted or restarted task skips finished batches) and
reports progress. All workers iterate the same number of times (ceil of the per-worker batch
count) so collectives inside ``process_batch`` never deadlock on uneven shards.
Off-cluster it runs the same loop with local checkpoint storage.
"""
import abc
import contextlib
import json
import logging
import math
import pathlib
import uuid
from typing import Any, Dict, Iterator, Optional, Type

import torch
import torch.nn as nn
from torch.utils import data

from determined_clone_amd import _info, core
from determined_clone_amd.pytorch import _data
from determined_clone_amd.pytorch._reducer import _PyTorchReducerContext

logger = logging.getLogger("determined_clone_amd.pytorch.experimental")

DEFAULT_BATCH_SIZE = 1


class TorchBatchProcessorContext(_PyTorchReducerContext):
    def __init__(self, core_context: Any, storage_path: str) -> None:
        super().__init__(core_context.distributed.allgather)
        self._core = core_context
        self.distributed = core_context.distributed
        self._storage_path = storage_path
        self.device = get_default_device(core_context)
        self._tensorboard_path: Optional[pathlib.Path] = None

    def get_hparams(self) -> Dict[str, Any]:
        info = _info.get_cluster_info()
        return dict(info.trial.hparams) if info and info.trial else {}

    def to_device(self, data_: Any, warned_types: Optional[set] = None) -> Any:
        return _data.to_device(data_, self.device, warned_types)

    def get_tensorboard_path(self) -> pathlib.Path:
        if self._tensorboard_path is None:
            self._tensorboard_path = self._core.train.get_tensorboard_path()
        return self._tensorboard_path

    def prepare_model_for_inference(self, model: nn.Module) -> nn.Module:
        """Move to this worker's device, eval mode, no grad; conv nets go channels_last."""
        model.eval()
        model = model.to(self.device)
        if self.device.type == "cuda" and any(isinstance(m, nn.Conv2d) for m in model.modules()):
            model = model.to(memory_format=torch.channels_last)
        for p in model.parameters():
            p.requires_grad_(False)
        return model

    @contextlib.contextmanager
    def upload_path(self) -> Iterator[pathlib.Path]:
        """Files written under the yielded path land in this worker's folder
        ``<default_output_uuid>/rank_<r>/`` of checkpoint storage. They are job OUTPUT, not
        checkpoints: nothing is registered with the master, so checkpoint GC never removes them
        (the resume-state checkpoints record ``default_output_uuid``)."""
        out_id, sub = self._storage_path.split("/", 1)
        with self._core.checkpoint._storage_manager.store_path(out_id) as p:
            out = pathlib.Path(p) / sub
            out.mkdir(parents=True, exist_ok=True)
            yield out

    def report_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any]) -> None:
        if self.distributed.rank != 0:
            return
        if group == "training":
            self._core.train.report_training_metrics(steps_completed, metrics)
        elif group == "validation":
            self._core.train.report_validation_metrics(steps_completed, metrics)
        else:
            self._core.train._report_metrics(group, steps_completed, metrics) \
                if hasattr(self._core.train, "_report_metrics") else \
                self._core.train.report_training_metrics(steps_completed, {f"{group}_{k}": v for k, v in metrics.items()})

    def report_task_using_model_version(self, model_version: Any) -> None:
        self._report_using(model_version.checkpoint.uuid if model_version.checkpoint else None)

    def report_task_using_checkpoint(self, checkpoint: Any) -> None:
        self._report_using(checkpoint.uuid)

    def _report_using(self, ckpt_uuid: Optional[str]) -> None:
        exp = getattr(self._core, "experimental", None)
        if ckpt_uuid and exp is not None and hasattr(exp, "report_task_using_checkpoint"):
            exp.report_task_using_checkpoint(ckpt_uuid)

    def get_distributed_rank(self) -> int:
        return self.distributed.rank

    def get_distributed_size(self) -> int:
        return self.distributed.size


def get_default_device(core_context: Any) -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", core_context.distributed.local_rank % torch.cuda.device_count())
    return torch.device("cpu")


class TorchBatchProcessor(metaclass=abc.ABCMeta):
    def __init__(self, context: TorchBatchProcessorContext) -> None:
        pass

    @abc.abstractmethod
    def process_batch(self, batch: Any, batch_idx: int) -> None:
        pass

    def on_checkpoint_start(self) -> None:
        """Called right before progress is checkpointed: flush buffered outputs here."""

    def on_finish(self) -> None:
        """Called once after the last batch on every worker."""


def _iterations(dataset_len: int, batch_size: int, workers: int, max_batches: Optional[int]) -> int:
    n = math.ceil(dataset_len / batch_size / workers)
    if max_batches is not None:
        if max_batches <= 0:
            raise ValueError("max_batches must be positive")
        n = min(n, max_batches)
    return n


def torch_batch_process(batch_processor_cls: Type[TorchBatchProcessor], dataset: data.Dataset,
                        batch_size: Optional[int] = None, max_batches: Optional[int] = None,
                        checkpoint_interval: int = 5, dataloader_kwargs: Optional[Dict[str, Any]] = None,
                        distributed_context: Optional[Any] = None) -> None:
    if checkpoint_interval <= 0:
        raise ValueError("checkpoint_interval should be a positive integer")
    dataloader_kwargs = dict(dataloader_kwargs or {})
    for k in ("shuffle", "sampler", "batch_sampler"):
        if k in dataloader_kwargs:
            raise ValueError(f"dataloader_kwargs may not set '{k}' (the dataset is sharded in order)")
    if batch_size is None:
        batch_size = int(dataloader_kwargs.pop("batch_size", DEFAULT_BATCH_SIZE))
    elif "batch_size" in dataloader_kwargs:
        raise ValueError("batch_size given twice (argument and dataloader_kwargs)")
    if not hasattr(dataset, "__len__"):
        raise TypeError("dataset must implement __len__()")
    if distributed_context is None:
        import os

        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            distributed_context = core.DistributedContext.from_torch_distributed()
    with core.init(distributed=distributed_context) as core_context:
        dist = core_context.distributed
        rank, workers = dist.rank, dist.size
        info = _info.get_cluster_info()
        skip = 0
        out_uuid = dist.broadcast(str(uuid.uuid4()) if rank == 0 else None)
        latest = info.latest_checkpoint if info else None
        if latest is not None:
            with core_context.checkpoint.restore_path(latest) as path:
                meta = json.loads((pathlib.Path(path) / "batch_process_state.json").read_text())
            skip = int(meta["steps_completed"])
            out_uuid = meta["default_output_uuid"]
            logger.info(f"resuming batch processing after {skip} batches")
        ctx = TorchBatchProcessorContext(core_context, f"{out_uuid}/rank_{rank}")
        processor = batch_processor_cls(ctx)
        loader = _data.DataLoader(dataset, batch_size=batch_size, shuffle=False, **dataloader_kwargs)
        it = iter(loader.get_data_loader(repeat=False, skip=skip, num_replicas=workers, rank=rank))
        n_iter = _iterations(len(dataset), batch_size, workers, max_batches)
        # the chief holds the trial's searcher operation (a dummy off-cluster): progress is reported
        # as a fraction of its length and it is completed at the end, so the experiment finishes
        ops = core_context.searcher.operations(core.SearcherMode.ChiefOnly) if rank == 0 else None
        op = next(ops, None) if ops is not None else None
        last_ckpt = -1
        batch_idx = skip - 1
        for batch_idx in range(skip, n_iter):
            batch = next(it, None)
            if batch is not None:
                processor.process_batch(batch=batch, batch_idx=batch_idx)
            if (batch_idx + 1) % checkpoint_interval == 0:
                processor.on_checkpoint_start()
                _checkpoint(core_context, batch_idx + 1, out_uuid)
                last_ckpt = batch_idx
                if op is not None:
                    op.report_progress(op.length * min(1.0, (batch_idx + 1) * batch_size * workers
                                                       / max(len(dataset), 1)))
                if core_context.preempt.should_preempt():
                    _reduce(ctx, core_context, rank, batch_idx + 1)
                    return
        if batch_idx > last_ckpt and batch_idx >= skip:
            processor.on_checkpoint_start()
            _checkpoint(core_context, batch_idx + 1, out_uuid)
        processor.on_finish()
        _reduce(ctx, core_context, rank, batch_idx + 1)
        if op is not None:
            op.report_completed(0.0)
            next(ops, None)  # out of operations: the trial is done


def _checkpoint(core_context: Any, steps_completed: int, out_uuid: str) -> None:
    dist = core_context.distributed
    dist.allgather(None)  # every worker finished the same batches
    if dist.rank == 0:
        with core_context.checkpoint.store_path({"steps_completed": steps_completed}) as (path, _sid):
            (pathlib.Path(path) / "batch_process_state.json").write_text(json.dumps(
                {"steps_completed": steps_completed, "default_output_uuid": out_uuid}))


def _reduce(ctx: TorchBatchProcessorContext, core_context: Any, rank: int, steps_completed: int) -> None:
    metrics = ctx.reduce_metrics(for_training=False)
    if rank == 0 and metrics:
        core_context.train.report_validation_metrics(steps_completed, metrics)
