"""The PyTorchTrial training loop (reference: `_PyTorchTrialController`,
`harness/determined/pytorch/_pytorch_trial.py:183-1413`).

Behaviour parity: searcher operations drive absolute training lengths; TRAIN / VALIDATE /
CHECKPOINT / REPORT boundaries in Batch or Epoch units (ints = periods, containers = schedules);
checkpoint policy best/all/none; preemption checked after each boundary; resume from
``latest_checkpoint`` restores model/optimizer/scheduler/scaler/callbacks/RNG and skips the batches
already trained; InvalidHP -> early exit.

MI355X-specific loop mechanics:
* the next batch is copied host->HBM on a side stream while the current step runs
  (`_data.DevicePrefetcher`);
* per-batch training metrics stay on the device until a boundary, where they are averaged across
  ranks with one collective and copied once (the reference syncs the GPU every batch);
* BN running statistics are broadcast from rank 0 only before validation/checkpoints.

Checkpoint format: ``state_dict.pth`` (models_state_dict, optimizers_state_dict,
lr_schedulers_state_dict, callbacks, rng_state, scaler_state_dict), ``load_data.json`` and
``trial_state.json``; all loadable with ``torch.load(weights_only=True)``.
"""
import contextlib
import json
import logging
import os
import pathlib
import random
import sys
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import numpy as np
import torch

from determined_clone_amd import profiler as profiler_mod
from determined_clone_amd import core, errors, util
from determined_clone_amd.ops import _grad
from determined_clone_amd.pytorch import _data, _reducer
from determined_clone_amd.pytorch._callback import PyTorchCallback
from determined_clone_amd.pytorch._trial import Batch, Epoch, PyTorchTrial, TrainUnit

logger = logging.getLogger("determined_clone_amd.pytorch")


class _BoundaryType:
    CHECKPOINT = "CHECKPOINT"
    REPORT = "REPORT"
    VALIDATE = "VALIDATE"
    TRAIN = "TRAIN"


class _Boundary:
    def __init__(self, step_type: str, unit: TrainUnit) -> None:
        self.step_type = step_type
        self.unit = unit
        self.limit_reached = False


class ShouldExit(Exception):
    def __init__(self, skip_exit_checkpoint: bool = False) -> None:
        self.skip_exit_checkpoint = skip_exit_checkpoint


class _TrialState:
    def __init__(self, trial_id: int = 0, last_ckpt: int = 0, step_id: int = 0, last_val: int = 0,
                 batches_trained: int = 0, epochs_trained: int = 0) -> None:
        self.trial_id = trial_id
        self.last_ckpt = last_ckpt
        self.step_id = step_id
        self.last_val = last_val
        self.batches_trained = batches_trained
        self.epochs_trained = epochs_trained


def _rng_state(local_rank: int) -> Dict[str, Any]:
    np_state = np.random.get_state()
    st: Dict[str, Any] = {
        "cpu_rng_state": torch.random.get_rng_state(),
        "np_rng_state": {"kind": np_state[0], "keys": torch.from_numpy(np_state[1].astype(np.int64)),
                         "pos": int(np_state[2]), "has_gauss": int(np_state[3]),
                         "cached_gaussian": float(np_state[4])},
        "random_rng_state": _py_random_state(),
    }
    if torch.cuda.is_available() and torch.cuda.device_count():
        st["gpu_rng_state"] = torch.cuda.get_rng_state(local_rank % torch.cuda.device_count())
    return st


def _py_random_state() -> Dict[str, Any]:
    version, internal, gauss = random.getstate()
    return {"version": version, "internal": list(internal), "gauss": gauss}


def _set_rng_state(st: Dict[str, Any], local_rank: int) -> None:
    if "cpu_rng_state" in st:
        torch.random.set_rng_state(st["cpu_rng_state"])
    nps = st.get("np_rng_state")
    if isinstance(nps, dict):
        np.random.set_state((nps["kind"], nps["keys"].numpy().astype(np.uint32), nps["pos"],
                             nps["has_gauss"], nps["cached_gaussian"]))
    elif isinstance(nps, (tuple, list)):
        np.random.set_state(tuple(nps))
    rs = st.get("random_rng_state")
    if isinstance(rs, dict):
        random.setstate((rs["version"], tuple(rs["internal"]), rs["gauss"]))
    elif isinstance(rs, (tuple, list)):
        random.setstate(tuple(rs))
    if "gpu_rng_state" in st and torch.cuda.is_available() and torch.cuda.device_count():
        torch.cuda.set_rng_state(st["gpu_rng_state"], local_rank % torch.cuda.device_count())


def load_state_dict_file(path: str) -> Dict[str, Any]:
    """Restricted unpickling only: weights_only=True, with numpy's array reconstructor allowed so
    reference-format checkpoints (raw numpy RNG state) also load."""
    try:
        return torch.load(path, map_location="cpu", weights_only=True)
    except Exception:
        safe = [np.core.multiarray._reconstruct, np.ndarray, np.dtype]
        try:
            safe.append(type(np.dtype("uint32")))
        except Exception:  # pragma: no cover
            pass
        with torch.serialization.safe_globals(safe):
            return torch.load(path, map_location="cpu", weights_only=True)


class _PyTorchTrialController:
    def __init__(self, trial_inst: PyTorchTrial, context: Any, checkpoint_period: TrainUnit,
                 validation_period: TrainUnit, reporting_period: TrainUnit,
                 smaller_is_better: bool, steps_completed: int, latest_checkpoint: Optional[str],
                 local_training: bool, test_mode: bool, searcher_metric_name: Optional[str],
                 checkpoint_policy: str, step_zero_validation: bool,
                 max_length: Optional[TrainUnit], global_batch_size: Optional[int],
                 profiler: Any = None) -> None:
        if not isinstance(trial_inst, self._trial_base()):
            raise TypeError(f"{type(self).__name__} requires a {self._trial_base().__name__}.")
        self.trial = trial_inst
        self.context = context
        self.core_context = context._core
        # Determined profiler (system metrics + loop timings, profiler.py); a no-op agent when
        # profiling is off. Timings end at a device synchronisation (reference
        # _pytorch_trial.py:200-209, 257).
        self.prof = profiler if profiler is not None else profiler_mod.DummyProfilerAgent()
        if torch.cuda.is_available():
            self.prof._set_sync_device(torch.cuda.synchronize)
        self.local_training = local_training
        self.is_chief = context.distributed.rank == 0
        self.max_length = max_length
        self.checkpoint_period = checkpoint_period
        self.validation_period = validation_period
        self.reporting_period = reporting_period
        if local_training:
            self.trial_id = 0
            if not self.max_length:
                raise ValueError("max_length must be specified for local-training mode.")
            self.searcher_unit = self.max_length._to_searcher_unit()
        else:
            self.trial_id = self.core_context.train._trial_id
            units = self.core_context.searcher.get_configured_units()
            if units is None:
                raise ValueError("Searcher units must be configured for training with PyTorchTrial.")
            self.searcher_unit = units
        self.state: Optional[_TrialState] = None
        self.start_from_batch = steps_completed
        self.val_from_previous_run = self.core_context.train._get_last_validation()
        self.step_zero_validation = step_zero_validation
        self.latest_checkpoint = latest_checkpoint
        self.test_mode = test_mode
        self.searcher_metric_name = searcher_metric_name
        self.ckpt_policy = checkpoint_policy
        self.smaller_is_better = smaller_is_better
        self.global_batch_size = global_batch_size
        if self.searcher_unit == core.Unit.RECORDS and self.global_batch_size is None:
            raise ValueError("global_batch_size required for searcher unit RECORDS.")
        self.callbacks: Dict[str, PyTorchCallback] = self.trial.build_callbacks()
        self._check_trial()
        self.last_step_time_s: float = 0.0
        self.samples_per_second: List[float] = []

    def _trial_base(self) -> type:
        return PyTorchTrial

    # Checkpoints written by every rank into one storage id (ZeRO shards); chief-only otherwise.
    _sharded_checkpoint = False

    def _check_trial(self) -> None:
        if len(self.context.models) == 0:
            raise errors.InvalidExperimentException(
                "Must have at least one model. This might be caused by not wrapping your model "
                "with wrap_model().")
        if len(self.context.optimizers) == 0:
            raise errors.InvalidExperimentException(
                "Must have at least one optimizer. This might be caused by not wrapping your "
                "optimizer with wrap_optimizer().")
        if self._evaluate_batch_defined() == self._evaluate_full_dataset_defined():
            raise errors.InvalidExperimentException(
                "Please define exactly one of: `evaluate_batch()` or `evaluate_full_dataset()`.")

    # ------------------------------------------------------------------ helpers
    def _evaluate_batch_defined(self) -> bool:
        return util.is_overridden(self.trial.evaluate_batch, PyTorchTrial)

    def _evaluate_full_dataset_defined(self) -> bool:
        return util.is_overridden(self.trial.evaluate_full_dataset, PyTorchTrial)

    def _set_data_loaders(self) -> None:
        skip = self.start_from_batch
        n, rank = self.context.distributed.size, self.context.distributed.rank
        train_data = self.trial.build_training_data_loader()
        if isinstance(train_data, _data.DataLoader):
            self.training_loader = train_data.get_data_loader(repeat=True, skip=skip, num_replicas=n, rank=rank)
        else:
            if self.context.experimental._data_repro_checks:
                raise RuntimeError(
                    "build_training_data_loader() returned a non-Determined DataLoader; call "
                    "context.experimental.disable_dataset_reproducibility_checks() to allow it")
            self.training_loader = train_data
        try:
            epoch_len = len(self.training_loader)
        except TypeError:
            epoch_len = sys.maxsize
        self.context._epoch_len = self.context.distributed.broadcast(epoch_len)
        self.validation_loader = None
        val_data = self.trial.build_validation_data_loader()
        if self._evaluate_batch_defined():
            if isinstance(val_data, _data.DataLoader):
                self.validation_loader = val_data.get_data_loader(repeat=False, skip=0, num_replicas=n, rank=rank)
            else:
                if self.context.experimental._data_repro_checks:
                    raise RuntimeError("build_validation_data_loader() returned a non-Determined DataLoader")
                self.validation_loader = val_data
        elif self.is_chief:
            self.validation_loader = (val_data.get_data_loader(repeat=False, skip=0, num_replicas=1, rank=0)
                                      if isinstance(val_data, _data.DataLoader) else val_data)

    def _checkpoint_is_current(self) -> bool:
        return self.state.last_ckpt == self.state.batches_trained

    def _validation_is_current(self) -> bool:
        return self.state.last_val == self.state.batches_trained

    def _steps_until_complete(self, unit: TrainUnit) -> int:
        assert isinstance(unit.value, int)
        if isinstance(unit, Batch):
            return unit.value - self.state.batches_trained
        if isinstance(unit, Epoch):
            return unit.value - self.state.epochs_trained
        raise ValueError(f"Unrecognized train unit {unit}")

    def _is_best_validation(self, now: float, before: Optional[float]) -> bool:
        if before is None:
            return True
        return (now < before) if self.smaller_is_better else (now > before)

    # ------------------------------------------------------------------ run
    @contextlib.contextmanager
    def _profiling(self) -> Iterator[None]:
        """The Determined profiler and the user's torch profiler (``context.set_profiler``) are
        entered ONCE around the training loop; the torch profiler's schedule advances with one
        ``step()`` per batch (``_train_batch``)."""
        with contextlib.ExitStack() as stack:
            stack.enter_context(self.prof)
            if self.context.profiler:
                stack.enter_context(self.context.profiler)
            yield

    def _timed_callback(self, name: str, fn: Any) -> Any:
        def call(*a: Any, **kw: Any) -> Any:
            with self.prof.record_timing(name):
                return fn(*a, **kw)
        return call

    def _timed_iter(self, it: Iterator[Any]) -> Iterator[Any]:
        """``next()`` of the training loader timed as ``dataloader_next`` (reference
        _pytorch_trial.py:34-40)."""
        while True:
            with self.prof.record_timing("dataloader_next", requires_sync=False):
                try:
                    item = next(it)
                except StopIteration:
                    return
            yield item

    def run(self) -> None:
        with contextlib.ExitStack() as stack:
            for name, cb in self.callbacks.items():
                cls = type(cb).__name__
                self._timed_callback(f"callbacks.{cls}.on_trial_startup", cb.on_trial_startup)(
                    self.start_from_batch, self.latest_checkpoint)
                stack.callback(self._timed_callback(f"callbacks.{cls}.on_trial_shutdown",
                                                    cb.on_trial_shutdown))
            if self.local_training and self.latest_checkpoint is not None:
                # Off-cluster there is no master to tell us steps_completed: take it from the
                # checkpoint so data loading resumes at the right batch.
                with self.core_context.checkpoint.restore_path(self.latest_checkpoint) as p:
                    st = p / "trial_state.json"
                    if st.exists():
                        self.start_from_batch = int(json.loads(st.read_text()).get("batches_trained", 0))
            self._set_data_loaders()
            util.startup_mark("data loaders built")
            it = iter(self.training_loader)
            if self.context.experimental._auto_to_device and self.context.device.type == "cuda":
                it = _data.DevicePrefetcher(it, self.context.device)
            self.training_iterator = it
            self.training_enumerator = enumerate(self._timed_iter(it), start=self.start_from_batch)
            util.startup_mark("training iterator ready")

            def cleanup() -> None:
                del self.training_iterator
                del self.training_enumerator

            stack.callback(cleanup)
            if self.latest_checkpoint is not None:
                logger.info(f"Restoring trial from checkpoint {self.latest_checkpoint}")
                with self.core_context.checkpoint.restore_path(self.latest_checkpoint) as load_path:
                    self._load(load_path)
            else:
                self.state = _TrialState(trial_id=self.trial_id)
            for cb in self.callbacks.values():
                cb.on_training_start()
            with _grad.step_stream(self.context.device), self._profiling():
                self._run()

    def _run(self) -> None:
        try:
            if self.step_zero_validation and self.val_from_previous_run is None and self.state.batches_trained == 0:
                self._validate()
            if self.local_training:
                ops: Iterator[Any] = iter([core.DummySearcherOperation(self.max_length.value, self.is_chief)])
            else:
                ops = self.core_context.searcher.operations()
            for op in ops:
                util.startup_mark("first searcher operation")
                train_unit = self.max_length if self.local_training else TrainUnit._from_searcher_unit(
                    op.length, self.searcher_unit, self.global_batch_size)
                self._train_for_op(op, [
                    _Boundary(_BoundaryType.TRAIN, train_unit),
                    _Boundary(_BoundaryType.VALIDATE, self.validation_period),
                    _Boundary(_BoundaryType.CHECKPOINT, self.checkpoint_period),
                    _Boundary(_BoundaryType.REPORT, self.reporting_period),
                ])
        except ShouldExit as e:
            if not e.skip_exit_checkpoint and not self._checkpoint_is_current():
                self._checkpoint(already_exiting=True)
        except errors.InvalidHP:
            if not self._checkpoint_is_current():
                self._checkpoint(already_exiting=True)
            raise

    def _train_with_boundaries(self, boundaries: List[_Boundary]) -> Tuple[List[_Boundary], List[Dict[str, Any]]]:
        metrics: List[Dict[str, Any]] = []
        if self.is_chief:
            self.core_context.train.set_status("training")
        self.prof.set_training(True)
        for m in self.context.models:
            m.train()
        self.context.reset_reducers()
        epoch_len = self.context._epoch_len
        for batch_idx, batch in self.training_enumerator:
            epoch_idx, in_epoch = divmod(batch_idx, epoch_len)
            self.context._current_batch_idx = batch_idx
            if in_epoch == 0:
                for cb in self.callbacks.values():
                    cb.on_training_epoch_start(epoch_idx)
            metrics.append(self._train_batch(batch, epoch_idx, batch_idx))
            self._step_batch()
            for b in boundaries:
                if isinstance(b.unit, Batch) and b.unit.should_stop(batch_idx + 1):
                    b.limit_reached = True
                if isinstance(b.unit, Epoch) and b.unit.should_stop(epoch_idx + 1) and in_epoch == epoch_len - 1:
                    b.limit_reached = True
                if b.step_type == _BoundaryType.TRAIN and self.test_mode:
                    b.limit_reached = True
            if any(b.limit_reached for b in boundaries):
                return boundaries, metrics
        return boundaries, metrics

    def _train_for_op(self, op: Any, boundaries: List[_Boundary]) -> None:
        if self.test_mode:
            length: TrainUnit = Batch(1)
        elif self.local_training:
            length = self.max_length
        else:
            length = TrainUnit._from_searcher_unit(op.length, self.searcher_unit, self.global_batch_size)
        while self._steps_until_complete(length) > 0:
            boundaries, batch_metrics = self._train_with_boundaries(boundaries)
            metrics = self._aggregate_training_metrics(batch_metrics)
            metrics = self.context.distributed.broadcast(metrics)
            for cb in self.callbacks.values():
                cb.on_training_workload_end(avg_metrics=metrics["avg_metrics"],
                                            batch_metrics=metrics["batch_metrics"])
            reported = False
            for b in boundaries:
                if not b.limit_reached:
                    continue
                if b.step_type in (_BoundaryType.TRAIN, _BoundaryType.REPORT):
                    if not op._completed and self.is_chief and not reported:
                        self._report_searcher_progress(op)
                        reported = True
                elif b.step_type == _BoundaryType.VALIDATE:
                    if not self._validation_is_current():
                        self._validate(op)
                elif b.step_type == _BoundaryType.CHECKPOINT:
                    if not self._checkpoint_is_current():
                        self._checkpoint(already_exiting=False)
                b.limit_reached = False
                self._stop_requested()
        if not self._validation_is_current():
            self._validate(op)
        if not self._checkpoint_is_current():
            self._checkpoint(already_exiting=False)
        if self.is_chief and not self.test_mode and not op._completed:
            raise ShouldExit(skip_exit_checkpoint=True)

    def _report_searcher_progress(self, op: Any) -> None:
        u = self.searcher_unit
        if u == core.Unit.BATCHES:
            op.report_progress(self.state.batches_trained)
        elif u == core.Unit.RECORDS:
            op.report_progress(self.global_batch_size * self.state.batches_trained)
        elif u == core.Unit.EPOCHS:
            op.report_progress(self.state.epochs_trained)

    def _stop_requested(self) -> None:
        if self.core_context.preempt.should_preempt():
            raise ShouldExit()
        if self.context.get_stop_requested():
            raise ShouldExit()

    def _step_batch(self) -> None:
        self.state.batches_trained += 1
        epoch_len = self.context._epoch_len
        epoch_idx, in_epoch = divmod(self.state.batches_trained - 1, epoch_len)
        if in_epoch == epoch_len - 1:
            for cb in self.callbacks.values():
                cb.on_training_epoch_end(epoch_idx)
            self.state.epochs_trained += 1

    def _auto_step_lr_scheduler_per_batch(self, batch_idx: int, sched: Any) -> None:
        if not self.context._should_communicate_and_update():
            return
        mode = sched._step_mode
        StepMode = type(sched).StepMode
        agg = self.context._aggregation_frequency
        if mode == StepMode.STEP_EVERY_BATCH:
            for i in range(batch_idx - agg + 1, batch_idx + 1):
                if (i + 1) % sched._frequency == 0:
                    sched.step()
        elif mode == StepMode.STEP_EVERY_OPTIMIZER_STEP:
            if (batch_idx + 1) % sched._frequency == 0:
                sched.step()
        elif mode == StepMode.STEP_EVERY_EPOCH:
            epoch_idx = batch_idx // self.context._epoch_len
            next_epoch = (batch_idx + agg) // self.context._epoch_len
            for e in range(epoch_idx, next_epoch):
                if (e + 1) % sched._frequency == 0:
                    sched.step()

    def _graph_step(self) -> Any:
        """The HIP-graph runner when ``optimizations.hip_graph`` is on and supported."""
        if not getattr(self.context, "_hip_graph", False):
            return None
        if getattr(self, "_graphed", None) is None:
            from determined_clone_amd.pytorch import _graph

            reason = _graph.unsupported_reason(self.context)
            if reason is not None:
                logger.warning(f"optimizations.hip_graph disabled: {reason}")
                self.context._hip_graph = False
                return None
            self._graphed = _graph.GraphedTrainStep(
                self.context, self.trial.train_batch, self.context._hip_graph_warmup,
                deterministic_convs=getattr(self.context, "_hip_graph_det_convs", False))
        return self._graphed

    _scratch_released = False

    def _release_first_step_scratch(self) -> None:
        """After the first training step, return the caching allocator's free blocks to the
        device once (``DCA_RELEASE_FIRST_STEP_SCRATCH``, default on): the first step carries
        one-off allocations -- the convolution chooser timing every candidate, MIOpen / GEMM
        workspaces, optimizer state creation -- that need not stay reserved for the rest of the
        trial. (The large reserved-vs-live gap of the round-3 bench came from elsewhere -- the
        side-stream gradients' record_stream, fixed in ops/_grad.py; see
        profiles/round4_bench_slow_mode.txt.)"""
        if self._scratch_released or self.context.device.type != "cuda":
            return
        self._scratch_released = True
        if os.environ.get("DCA_RELEASE_FIRST_STEP_SCRATCH", "1") != "0":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    def _train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        util.startup_mark("first batch fetched")
        self.context._loss_ids = {}
        t0 = time.time()
        self.prof.update_batch_idx(batch_idx)
        if self.context.experimental._auto_to_device and not isinstance(self.training_iterator, _data.DevicePrefetcher):
            with self.prof.record_timing("to_device", accumulate=True):
                batch = self.context.to_device(batch)
        with self.prof.record_timing("train_batch", requires_sync=False):
            if self.context.profiler:
                out = self.trial.train_batch(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
                self.context.profiler.step()
            elif self._graph_step() is not None:
                out = self._graphed(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
            else:
                out = self.trial.train_batch(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
        if self.context._scaler is not None and self.context.experimental._auto_amp \
                and self.context._should_communicate_and_update():
            self.context._scaler.update()
        util.startup_mark("first train batch")
        self._release_first_step_scratch()
        if isinstance(out, torch.Tensor):
            out = {"loss": out}
        if not isinstance(out, dict):
            raise TypeError("train_batch() must return a dictionary mapping string names to Tensor "
                            f"metrics, got {type(out).__name__}")
        with self.prof.record_timing("step_lr_schedulers"):
            for sched in self.context.lr_schedulers:
                self._auto_step_lr_scheduler_per_batch(batch_idx, sched)
        # metrics stay on the device until the workload's reduction (no per-batch host sync)
        with self.prof.record_timing("from_device"):
            metrics = {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
        dt = time.time() - t0
        self.last_step_time_s = dt
        if dt > 0:
            sps = self.trial.get_batch_length(batch) * self.context.distributed.size / dt
            self.samples_per_second.append(sps)
            self.prof.record_metric("samples_per_second", sps)
        return metrics

    def _aggregate_training_metrics(self, batch_metrics: List[Dict[str, Any]]) -> Dict[str, Any]:
        with self.prof.record_timing("average_training_metrics"):
            agg = _reducer.average_training_metrics(self.context.distributed, batch_metrics,
                                                    self.context._average_training_metrics)
        with self.prof.record_timing("reduce_metrics"):
            extra = self.context.reduce_metrics(for_training=True)
        agg["avg_metrics"].update({k: util.to_python(v) for k, v in extra.items()})
        if not self.is_chief:
            return {"avg_metrics": agg["avg_metrics"], "batch_metrics": agg["batch_metrics"]}
        self.core_context.train.report_training_metrics(
            steps_completed=self.state.batches_trained, metrics=agg["avg_metrics"],
            batch_metrics=agg["batch_metrics"])
        return agg

    @torch.no_grad()
    def _validate(self, searcher_op: Any = None) -> Dict[str, Any]:
        if self.is_chief:
            self.core_context.train.set_status("validating")
        self.context.reset_reducers()
        self.context._sync_buffers()
        # ZeRO overlap_param_gather: evaluation / metric code may read parameters directly
        # (p.data, tied weights) -- every in-flight all-gather lands first
        for o in list(getattr(self.context, "optimizers", [])) + list(self.context.models):
            wait = getattr(o, "wait_params", None)
            if callable(wait):
                wait()
        for m in self.context.models:
            m.eval()
        t0 = time.time()
        for cb in self.callbacks.values():
            cb.on_validation_start()
        metrics = self._compute_validation_metrics()
        util.startup_mark("first validation")
        metrics.update(self.context.reduce_metrics(for_training=False))
        metrics = {k: util.to_python(v) for k, v in metrics.items()}
        if self.context.distributed.size > 1:
            metrics = self.context.distributed.broadcast(metrics)
        for cb in self.callbacks.values():
            cb.on_validation_end(metrics)
        self.state.last_val = self.state.batches_trained
        best_before = None
        if self.is_chief:
            best_before = self.core_context.train.get_experiment_best_validation()
            self.core_context.train.report_validation_metrics(self.state.batches_trained, metrics)
            logger.info(f"validated in {time.time() - t0:.2f}s")
        searcher_metric = None
        if self.is_chief and searcher_op is not None:
            length = self.max_length if self.local_training else TrainUnit._from_searcher_unit(
                searcher_op.length, self.searcher_unit, self.global_batch_size)
            if self.searcher_metric_name:
                if self.searcher_metric_name not in metrics:
                    raise RuntimeError(f"Search method is configured to use metric "
                                       f"'{self.searcher_metric_name}' but the model returned "
                                       f"validation metrics {list(metrics)}")
                searcher_metric = metrics[self.searcher_metric_name]
                if not util.is_numerical_scalar(searcher_metric):
                    raise RuntimeError(f"Searcher validation metric '{self.searcher_metric_name}' "
                                       f"returned a non-scalar value: {searcher_metric}")
            if self._steps_until_complete(length) < 1 and not searcher_op._completed:
                searcher_op.report_completed(searcher_metric)
        should_ckpt = False
        if self.is_chief and not self._checkpoint_is_current():
            if self.ckpt_policy == "all":
                should_ckpt = True
            elif self.ckpt_policy == "best" and searcher_metric is not None:
                should_ckpt = self._is_best_validation(float(searcher_metric), best_before)
        should_ckpt = self.context.distributed.broadcast(should_ckpt)
        if should_ckpt:
            self._checkpoint(already_exiting=False)
        return metrics

    def _compute_validation_metrics(self) -> Dict[str, Any]:
        metrics: Dict[str, Any] = {}
        if self._evaluate_batch_defined():
            keys = None
            batch_metrics: List[Dict[str, Any]] = []
            if len(self.validation_loader) == 0:
                raise RuntimeError("validation_loader is empty.")
            for cb in self.callbacks.values():
                cb.on_validation_epoch_start()
            idx = -1
            for idx, batch in enumerate(iter(self.validation_loader)):
                if self.context.experimental._auto_to_device:
                    batch = self.context.to_device(batch)
                if util.has_param(self.trial.evaluate_batch, "batch_idx", 2):
                    vm = self.trial.evaluate_batch(batch=batch, batch_idx=idx)
                else:
                    vm = self.trial.evaluate_batch(batch=batch)
                if not isinstance(vm, dict):
                    raise TypeError(f"evaluate_batch() must return a dict, got {type(vm).__name__}")
                if keys is None:
                    keys = vm.keys()
                elif keys != vm.keys():
                    raise ValueError(f"Validation metric names must match across all batches: "
                                     f"{keys} != {vm.keys()}")
                batch_metrics.append({k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in vm.items()})
                if self.test_mode:
                    break
            for cb in self.callbacks.values():
                cb.on_validation_epoch_end(batch_metrics)
            metrics = _reducer.reduce_validation_metrics(
                self.context.distributed, batch_metrics, keys,
                _reducer._prepare_metrics_reducers(self.trial.evaluation_reducer(), keys=keys or []))
        else:
            if self.is_chief:
                metrics = self.trial.evaluate_full_dataset(data_loader=self.validation_loader)
                if not isinstance(metrics, dict):
                    raise TypeError(f"evaluate_full_dataset() must return a dict, got {type(metrics).__name__}")
        return metrics

    # ------------------------------------------------------------------ checkpoint
    def _checkpoint(self, already_exiting: bool) -> None:
        if os.environ.get("DET_STARTUP_PROFILE") == "checkpoint" and not getattr(self, "_ckpt_profiled", False):
            # start-up investigation: cProfile of the first checkpoint, into the task log
            import cProfile
            import io
            import pstats

            self._ckpt_profiled = True
            prof = cProfile.Profile()
            prof.enable()
            try:
                return self._checkpoint(already_exiting)
            finally:
                prof.disable()
                buf = io.StringIO()
                pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(30)
                logging.getLogger("determined_clone_amd.startup").info(buf.getvalue())
        if self.is_chief:
            self.core_context.train.set_status("checkpointing")
        self.state.last_ckpt = self.state.batches_trained
        self.context._sync_buffers()
        try:
            uuid = ""
            from determined_clone_amd import __version__

            md = {"determined_version": __version__,
                  "steps_completed": self.state.batches_trained,
                  "framework": f"torch-{torch.__version__}", "format": "pickle"}
            if self._sharded_checkpoint:
                with self.core_context.checkpoint.store_path(md if self.is_chief else {}, shard=True) as (path, storage_id):
                    self._save(path)
                    uuid = storage_id
            elif self.is_chief:
                with self.core_context.checkpoint.store_path(md) as (path, storage_id):
                    self._save(path)
                    uuid = storage_id
            uuid = self.context.distributed.broadcast(uuid)
            util.startup_mark("first checkpoint")
            for cb in self.callbacks.values():
                cb.on_checkpoint_upload_end(uuid=uuid)
        except errors.InvalidHP:
            if not already_exiting:
                self.core_context.train.report_early_exit(core.EarlyExitReason.INVALID_HP)
                raise ShouldExit(skip_exit_checkpoint=True)
            raise

    def _save(self, path: pathlib.Path) -> None:
        path.mkdir(parents=True, exist_ok=True)
        util.write_user_code(path, not self.local_training)
        for o in self.context.optimizers:  # ZeRO: parameter all-gathers may still be in flight
            wait = getattr(o, "wait_params", None)
            if wait is not None:
                wait()
        ckpt: Dict[str, Any] = {
            "models_state_dict": [m.state_dict() for m in self.context.models],
            "optimizers_state_dict": [o.state_dict() for o in self.context.optimizers],
            "lr_schedulers_state_dict": [s.state_dict() for s in self.context.lr_schedulers],
            "callbacks": {n: cb.state_dict() for n, cb in self.callbacks.items()},
            "rng_state": _rng_state(self.context.distributed.local_rank),
        }
        if self.context._scaler is not None:
            ckpt["scaler_state_dict"] = self.context._scaler.state_dict()
        for cb in self.callbacks.values():
            cb.on_checkpoint_save_start(ckpt)
        torch.save(ckpt, str(path / "state_dict.pth"))
        (path / "trial_state.json").write_text(json.dumps(vars(self.state)))
        try:
            exp_conf: Optional[Dict[str, Any]] = self.context.get_experiment_config()
            hparams: Optional[Dict[str, Any]] = self.context.get_hparams()
        except ValueError:
            exp_conf, hparams = None, None
        tc = type(self.trial)
        load_data = {"trial_type": "PyTorchTrial", "experiment_config": exp_conf,
                     "hparams": hparams, "trial_cls_spec": f"{tc.__module__}:{tc.__qualname__}",
                     "is_trainer": True}
        if self.context._is_pre_trainer:
            load_data.pop("is_trainer")
        (path / "load_data.json").write_text(json.dumps(load_data, default=str))
        for cb in self.callbacks.values():
            cb.on_checkpoint_end(str(path))
            cb.on_checkpoint_write_end(str(path))

    def _load(self, load_path: pathlib.Path) -> None:
        ckpt = None
        for rel in (["state_dict.pth"], ["determined", "state_dict.pth"], ["pedl", "state_dict.pth"], ["checkpoint.pt"]):
            p = load_path.joinpath(*rel)
            if p.exists():
                ckpt = load_state_dict_file(str(p))
                break
        if not isinstance(ckpt, dict):
            self.state = _TrialState(trial_id=self.trial_id)
            return
        for cb in self.callbacks.values():
            cb.on_checkpoint_load_start(ckpt)
        if "model_state_dict" in ckpt:
            if len(self.context.models) > 1:
                raise RuntimeError("Old-format checkpoint cannot be loaded into a context with more than one model.")
            self.context.models[0].load_state_dict(ckpt["model_state_dict"])
        else:
            for i, m in enumerate(self.context.models):
                sd = ckpt["models_state_dict"][i]
                try:
                    m.load_state_dict(sd)
                except RuntimeError:
                    torch.nn.modules.utils.consume_prefix_in_state_dict_if_present(sd, "module.")
                    m.load_state_dict(sd)
        osd = ckpt.get("optimizers_state_dict") or ([ckpt["optimizer_state_dict"]] if "optimizer_state_dict" in ckpt else [])
        for i, o in enumerate(self.context.optimizers):
            if i < len(osd):
                o.load_state_dict(osd[i])
        from determined_clone_amd.ops.optim import FusedOptimizerBase

        for o in self.context.optimizers:
            if isinstance(o, FusedOptimizerBase) and not any(
                    "master_param" in s for s in (osd[0]["state"].values() if osd else [])):
                o.sync_master_from_model()
        ssd = ckpt.get("lr_schedulers_state_dict") or ([ckpt["lr_scheduler"]] if "lr_scheduler" in ckpt else [])
        for i, s in enumerate(self.context.lr_schedulers):
            if i < len(ssd):
                s.load_state_dict(ssd[i])
        if "scaler_state_dict" in ckpt and self.context._scaler is not None:
            self.context._scaler.load_state_dict(ckpt["scaler_state_dict"])
        for name, cb in self.callbacks.items():
            if name in ckpt.get("callbacks", {}):
                cb.load_state_dict(ckpt["callbacks"][name])
        if "rng_state" in ckpt:
            _set_rng_state(ckpt["rng_state"], self.context.distributed.local_rank)
        st_path = load_path / "trial_state.json"
        if st_path.exists():
            st = json.loads(st_path.read_text())
            if st.get("trial_id") != self.trial_id:
                self.state = _TrialState(trial_id=self.trial_id)
            else:
                self.state = _TrialState(**st)
                if self.state.batches_trained == self.val_from_previous_run:
                    self.state.last_val = self.state.batches_trained
        else:
            self.state = _TrialState(trial_id=self.trial_id)
