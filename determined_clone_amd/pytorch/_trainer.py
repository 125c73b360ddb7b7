"""Trainer API: ``pytorch.init()`` + ``Trainer.fit()`` (reference: `harness/determined/pytorch/_trainer.py`)."""
import contextlib
import logging
import os
import random
import sys
from typing import Any, Dict, Iterator, Optional

import numpy as np
import torch

from determined_clone_amd import _info, core
from determined_clone_amd.pytorch._context import PyTorchTrialContext
from determined_clone_amd.pytorch._controller import _PyTorchTrialController
from determined_clone_amd.pytorch._trial import Batch, PyTorchTrial, TrainUnit

logger = logging.getLogger("determined_clone_amd.pytorch")


class Trainer:
    def __init__(self, trial: PyTorchTrial, context: PyTorchTrialContext) -> None:
        self._trial = trial
        self._context = context
        self._core = context._core
        self._info = _info.get_cluster_info()
        self._local_training = self._info is None or self._info.task_type != "TRIAL"
        self._profiler: Any = None

    def configure_profiler(self, enabled: bool = False, sync_timings: bool = True,
                           begin_on_batch: int = 0, end_after_batch: Optional[int] = None) -> None:
        """Configure the Determined profiler (reference pytorch/_trainer.py:36-84): on-cluster
        only; in local training it is a no-op. Samples system metrics (GPU utilisation / free
        VRAM from amdgpu sysfs, CPU, memory, network, disk) and the loop's timings between
        ``begin_on_batch`` and ``end_after_batch`` (at most 5 minutes) and ships them to the
        master's ``/api/v1/trials/profiler/metrics``."""
        from determined_clone_amd import profiler

        if self._local_training or self._info is None:
            self._profiler = profiler.DummyProfilerAgent()
            return
        session = getattr(self._core.train, "_session", None)
        self._profiler = profiler.ProfilerAgent.from_config(
            {"enabled": enabled, "sync_timings": sync_timings, "begin_on_batch": begin_on_batch,
             "end_after_batch": end_after_batch},
            trial_id=self._info.trial.trial_id, agent_id=self._info.agent_id,
            global_rank=self._core.distributed.get_rank(),
            local_rank=self._core.distributed.get_local_rank(), session=session)

    def fit(self, checkpoint_period: Optional[TrainUnit] = None,
            validation_period: Optional[TrainUnit] = None, max_length: Optional[TrainUnit] = None,
            reporting_period: TrainUnit = Batch(100),  # noqa: B008
            checkpoint_policy: str = "best", latest_checkpoint: Optional[str] = None,
            step_zero_validation: bool = False, test_mode: bool = False) -> Any:
        checkpoint_period = checkpoint_period or Batch(sys.maxsize)
        validation_period = validation_period or Batch(sys.maxsize)
        if self._local_training:
            if checkpoint_policy == "best":
                logger.warning("checkpoint_policy='best' is not supported in local training mode; using 'all'")
                checkpoint_policy = "all"
            if max_length is None:
                raise ValueError("max_length must be defined in local training mode.")
            if not isinstance(max_length.value, int):
                raise TypeError("max_length must be configured in TrainUnit(int) types.")
            smaller_is_better, metric_name, steps_completed, gbs = True, None, 0, None
        else:
            if test_mode:
                raise ValueError("test_mode is only supported in local training mode.")
            if max_length is not None:
                logger.warning("max_length is ignored when training on-cluster; configure the searcher instead")
            cfg = self._info.trial._config
            if latest_checkpoint is None and self._info.latest_checkpoint is not None:
                logger.warning("latest_checkpoint not passed to fit(); pause/resume will restart "
                               "from scratch. Did you mean fit(latest_checkpoint=info.latest_checkpoint)?")
            smaller_is_better = bool(cfg["searcher"]["smaller_is_better"])
            metric_name = cfg["searcher"]["metric"]
            steps_completed = int(self._info.trial._steps_completed)
            gbs = self._info.trial.hparams.get("global_batch_size")
            gbs = int(gbs) if gbs else None
        controller = _PyTorchTrialController(
            trial_inst=self._trial, context=self._context, checkpoint_period=checkpoint_period,
            validation_period=validation_period, reporting_period=reporting_period,
            smaller_is_better=smaller_is_better, steps_completed=steps_completed,
            latest_checkpoint=latest_checkpoint, local_training=self._local_training,
            test_mode=test_mode, searcher_metric_name=metric_name,
            checkpoint_policy=checkpoint_policy, step_zero_validation=step_zero_validation,
            max_length=max_length, global_batch_size=gbs, profiler=self._profiler)
        controller.run()
        return controller


def _initialize_distributed_backend() -> Optional[core.DistributedContext]:
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and "RANK" in os.environ:
        return core.DistributedContext.from_torch_distributed()
    info = _info.get_cluster_info()
    if info and (len(info.container_addrs) > 1 or len(info.slot_ids) > 1):
        raise ValueError("multi-slot training needs a distributed launch layer such as "
                         "determined_clone_amd.launch.torch_distributed")
    return None


def _set_random_seeds(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.random.manual_seed(seed)


@contextlib.contextmanager
def init(*, hparams: Optional[Dict] = None, exp_conf: Optional[Dict[str, Any]] = None,
         distributed: Optional[core.DistributedContext] = None, aggregation_frequency: int = 1,
         enable_tensorboard_logging: bool = True) -> Iterator[PyTorchTrialContext]:
    info = _info.get_cluster_info()
    local_training = info is None or info.task_type != "TRIAL"
    dist_ctx = distributed
    if local_training:
        seed, steps_completed, debug = None, 0, False
        num_gpus = torch.cuda.device_count() if torch.cuda.is_available() else 0
        if dist_ctx is None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            dist_ctx = _initialize_distributed_backend()
    else:
        dist_ctx = dist_ctx or _initialize_distributed_backend()
        seed = info.trial.trial_seed
        exp_conf = info.trial._config
        hparams = hparams if hparams is not None else info.trial.hparams
        steps_completed = info.trial._steps_completed
        num_gpus = len(info.gpu_uuids) or (torch.cuda.device_count() if torch.cuda.is_available() else 0)
        debug = info.trial._debug
        _set_random_seeds(seed)
        opts = (exp_conf or {}).get("optimizations", {}) or {}
        aggregation_frequency = int(opts.get("aggregation_frequency", aggregation_frequency))
    with core.init(distributed=dist_ctx, preempt_mode=core.PreemptMode.WorkersAskChief,
                   tensorboard_mode=core.TensorboardMode.MANUAL) as core_context:
        ctx = PyTorchTrialContext(core_context=core_context, trial_seed=seed, hparams=hparams,
                                  slots_per_trial=core_context.distributed.get_size(),
                                  num_gpus=num_gpus, exp_conf=exp_conf,
                                  aggregation_frequency=aggregation_frequency,
                                  steps_completed=steps_completed, managed_training=True,
                                  debug_enabled=debug,
                                  enable_tensorboard_logging=enable_tensorboard_logging)
        yield ctx
