"""DeepSpeedTrial / DeepSpeedTrialContext / controller on the native ZeRO engine.

Reference: `harness/determined/pytorch/deepspeed/_deepspeed_trial.py` (DeepSpeedTrialController:
micro-batch accumulation in ``_train_for_step``, iterator-style ``train_batch(dataloader_iter, ...)``
/ ``evaluate_batch(dataloader_iter, idx)``, per-rank ``det_state_dict_rank{r}.pth`` + every rank's
engine ``save_checkpoint`` into one sharded checkpoint) and `_deepspeed_context.py`
(wrap_model_engine, set_mpu, disable_auto_grad_accumulation, overwrite_deepspeed_config).

Differences by design: the engine is :class:`~._engine.DeepSpeedEngine` (native ZeRO-1/2 on RCCL,
no DeepSpeed/apex dependency); data loaders are skipped by ``steps_completed * micro_batches``
micro-batches on resume; checkpoints are written with ``weights_only``-loadable content.
"""
import abc
import contextlib
import json
import logging
import os
import pathlib
import sys
import time
from typing import Any, Dict, Iterator, List, Optional, Union

import torch

from determined_clone_amd.ops import _grad
from determined_clone_amd import _info, core, errors, util
from determined_clone_amd.pytorch import _data, _reducer
from determined_clone_amd.pytorch._callback import PyTorchCallback
from determined_clone_amd.pytorch._context import PyTorchTrialContext
from determined_clone_amd.pytorch._controller import (_PyTorchTrialController, _rng_state,
                                                      _set_rng_state, _TrialState,
                                                      load_state_dict_file)
from determined_clone_amd.pytorch._trial import Batch, TrainUnit
from determined_clone_amd.pytorch.deepspeed._engine import DeepSpeedEngine
from determined_clone_amd.pytorch.deepspeed._mpu import (ModelParallelUnit, make_data_parallel_mpu,
                                                         make_deepspeed_mpu)
from determined_clone_amd.pytorch.dsat import _defaults as dsat_defaults

logger = logging.getLogger("determined_clone_amd.pytorch.deepspeed")


def overwrite_deepspeed_config(base_ds_config: Union[str, Dict[str, Any]],
                               source_ds_dict: Dict[str, Any]) -> Dict[str, Any]:
    """Overwrite leaves of a DeepSpeed config (path or dict) with ``source_ds_dict``
    (reference `_deepspeed_context.py:19`)."""
    if isinstance(base_ds_config, str):
        with open(base_ds_config) as f:
            base_ds_config = json.load(f)
    elif not isinstance(base_ds_config, dict):
        raise TypeError("Expected string or dict for base_ds_config argument.")
    return util.merge_dicts(base_ds_config, source_ds_dict)


class DeepSpeedTrialContext(PyTorchTrialContext):
    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        opts = (self._exp_conf or {}).get("optimizations", {}) or {}
        if opts.get("mixed_precision", "O0") != "O0":
            raise errors.InvalidExperimentException(
                "Mixed precision is specified through the deepspeed config instead of the "
                "Determined experiment config.")
        if int(opts.get("aggregation_frequency", 1)) > 1:
            raise errors.InvalidExperimentException(
                "Gradient aggregation is specified through the deepspeed config instead of the "
                "Determined experiment config.")
        self._average_training_metrics = bool(opts.get("average_training_metrics", False))
        self._mpu = make_data_parallel_mpu(self.distributed)
        self._called_set_mpu = False
        self._train_micro_batch_size_per_gpu: Optional[int] = None
        self._num_micro_batches_per_slot: Optional[int] = None
        self._use_pipeline_parallel = False
        self._manual_grad_accumulation = False

    def set_mpu(self, mpu: ModelParallelUnit) -> None:
        if not self.models:
            raise errors.InvalidExperimentException("Please call `wrap_model_engine` before setting the mpu.")
        if self._called_set_mpu:
            raise errors.InvalidExperimentException("Only one MPU can be passed to DeepSpeedTrialContext.")
        if self.distributed.rank == 0 and not mpu.should_report_metrics and not self._average_training_metrics:
            raise errors.InvalidExperimentException(
                "Please set optimizations.average_training_metrics in the experiment config to true "
                "so that metrics will exist on the chief for report to the master.")
        self._called_set_mpu = True
        self._mpu = mpu

    def wrap_model_engine(self, model: DeepSpeedEngine) -> DeepSpeedEngine:
        model = model.to(self.device)
        from determined_clone_amd.pytorch.deepspeed._pipe import PipelineEngine

        if isinstance(model, PipelineEngine):
            # the pipeline engine's stage x data grid defines the data-parallel coordinates
            # (reference: _deepspeed_context.py:188)
            self._use_pipeline_parallel = True
            if not self.models:
                self._mpu = make_deepspeed_mpu(model.grid)
            else:
                logger.warning("Using the MPU corresponding to the first wrapped model engine.")
        if not self.models:
            self._train_micro_batch_size_per_gpu = int(model.train_micro_batch_size_per_gpu())
            self._num_micro_batches_per_slot = int(model.gradient_accumulation_steps())
        elif model.train_micro_batch_size_per_gpu() != self._train_micro_batch_size_per_gpu:
            logger.warning(f"Train micro batch size for wrapped model engine {len(self.models) + 1} "
                           "does not match that of the first wrapped engine.")
        self.models.append(model)
        return model

    def disable_auto_grad_accumulation(self) -> None:
        self._manual_grad_accumulation = True

    def disable_dataset_reproducibility_checks(self) -> None:
        self.experimental.disable_dataset_reproducibility_checks()

    @property
    def use_pipeline_parallel(self) -> bool:
        return self._use_pipeline_parallel

    @property
    def train_micro_batch_size_per_gpu(self) -> int:
        if self._train_micro_batch_size_per_gpu is None:
            raise errors.InvalidExperimentException(
                "Please call wrap_model_engine before accessing train_micro_batch_size.")
        return self._train_micro_batch_size_per_gpu

    @property
    def num_micro_batches_per_slot(self) -> int:
        if self._num_micro_batches_per_slot is None:
            raise errors.InvalidExperimentException(
                "Please call wrap_model_engine before accessing num_micro_batches_per_slot.")
        return self._num_micro_batches_per_slot

    def _sync_buffers(self) -> None:
        from determined_clone_amd.parallel import ddp
        from determined_clone_amd.pytorch.deepspeed._pipe import PipelineEngine

        for m in self.models:
            mod = m.module if isinstance(m, DeepSpeedEngine) else m
            if self.distributed.size > 1:
                group, src = None, 0
                if isinstance(m, PipelineEngine):
                    # stages hold different layers: buffers are synced within a stage's replicas
                    if m.grid.data_parallel_size == 1:
                        continue
                    group, src = m.grid.dp_group, m.grid.stage_to_global(m.stage_id, 0)
                bufs = list(mod.buffers())
                if bufs:
                    ddp._broadcast_coalesced(bufs, group, src)


class DeepSpeedTrial(metaclass=abc.ABCMeta):
    """Subclass and build a :class:`DeepSpeedEngine` (``det_ds.initialize``) in ``__init__``, then
    ``context.wrap_model_engine(engine)``. ``train_batch`` receives the training ITERATOR and is
    called ``gradient_accumulation_steps`` times per batch unless auto accumulation is disabled."""

    trial_context_class = DeepSpeedTrialContext
    _is_deepspeed_trial = True

    @abc.abstractmethod
    def __init__(self, context: DeepSpeedTrialContext) -> None:
        pass

    @abc.abstractmethod
    def train_batch(self, dataloader_iter: Optional[Iterator[Any]], epoch_idx: int,
                    batch_idx: int) -> Union[torch.Tensor, Dict[str, Any]]:
        pass

    @abc.abstractmethod
    def build_training_data_loader(self) -> Any:
        pass

    @abc.abstractmethod
    def build_validation_data_loader(self) -> Any:
        pass

    def build_callbacks(self) -> Dict[str, PyTorchCallback]:
        return {}

    @abc.abstractmethod
    def evaluate_batch(self, dataloader_iter: Optional[Iterator[Any]], batch_idx: int) -> Dict[str, Any]:
        pass

    def evaluation_reducer(self) -> Any:
        return _reducer.Reducer.AVG

    def save(self, context: DeepSpeedTrialContext, path: pathlib.Path) -> None:
        for i, m in enumerate(context.models):
            m.save_checkpoint(path, tag=f"model{i}")

    def load(self, context: DeepSpeedTrialContext, load_path: pathlib.Path) -> None:
        for i, m in enumerate(context.models):
            m.load_checkpoint(load_path, tag=f"model{i}")

    def get_batch_length(self, batch: Any) -> int:
        return _data.data_length(batch)


class DeepSpeedTrialController(_PyTorchTrialController):
    _sharded_checkpoint = True

    def _trial_base(self) -> type:
        return DeepSpeedTrial

    def _check_trial(self) -> None:
        if not self.context.models:
            raise errors.InvalidExperimentException(
                "Must have at least one model engine. This might be caused by not wrapping your "
                "model with wrap_model_engine()")

    def _evaluate_batch_defined(self) -> bool:
        return True

    def _evaluate_full_dataset_defined(self) -> bool:
        return False

    # ------------------------------------------------------------------ data
    def _set_data_loaders(self) -> None:
        ctx = self.context
        mpu = ctx._mpu
        nmb = ctx.num_micro_batches_per_slot
        skip = self.start_from_batch * (1 if ctx._manual_grad_accumulation else nmb)
        self.training_loader = None
        self.validation_loader = None
        self.num_validation_batches: Optional[int] = None
        n, rank = mpu.data_parallel_world_size, mpu.data_parallel_rank
        if mpu.should_build_data_loader:
            td = self.trial.build_training_data_loader()
            if isinstance(td, _data.DataLoader):
                self.training_loader = td.get_data_loader(repeat=True, skip=skip, num_replicas=n, rank=rank)
            else:
                if ctx.experimental._data_repro_checks:
                    raise RuntimeError("build_training_data_loader() returned a non-Determined "
                                       "DataLoader; call context.disable_dataset_reproducibility_checks()")
                self.training_loader = td
            vd = self.trial.build_validation_data_loader()
            if isinstance(vd, _data.DataLoader):
                self.validation_loader = vd.get_data_loader(repeat=False, skip=0, num_replicas=n, rank=rank)
            else:
                if ctx.experimental._data_repro_checks:
                    raise RuntimeError("build_validation_data_loader() returned a non-Determined "
                                       "DataLoader; call context.disable_dataset_reproducibility_checks()")
                self.validation_loader = vd
            self.num_validation_batches = len(self.validation_loader)
            if ctx.use_pipeline_parallel:
                # each evaluate_batch call runs one pipelined eval over nmb micro-batches
                # (reference: _deepspeed_trial.py:155)
                if self.num_validation_batches < nmb:
                    raise errors.InvalidExperimentException(
                        "Number of train micro batches in validation data loader should not be less "
                        "than the number of gradient accumulation steps when using pipeline "
                        "parallelism.")
                self.num_validation_batches //= nmb
        try:
            elen = len(self.training_loader) if self.training_loader is not None else None
        except TypeError:
            elen = sys.maxsize
        all_lens = [x for x in ctx.distributed.allgather(elen) if x is not None]
        ctx._epoch_len = max(1, min(all_lens) // (1 if ctx._manual_grad_accumulation else nmb))
        all_val = [x for x in ctx.distributed.allgather(self.num_validation_batches) if x is not None]
        self.num_validation_batches = min(all_val) if all_val else 0

    def run(self) -> None:
        # The base run() wraps the training loader in an enumerator/prefetcher; DeepSpeedTrial hands
        # the raw iterator to train_batch instead.
        with contextlib.ExitStack() as stack:
            for cb in self.callbacks.values():
                cb.on_trial_startup(self.start_from_batch, self.latest_checkpoint)
                stack.callback(cb.on_trial_shutdown)
            if self.local_training and self.latest_checkpoint is not None:
                with self.core_context.checkpoint.restore_path(self.latest_checkpoint) as p:
                    st = p / "trial_state.json"
                    if st.exists():
                        self.start_from_batch = int(json.loads(st.read_text()).get("batches_trained", 0))
            self._set_data_loaders()
            self.training_iterator = iter(self.training_loader) if self.training_loader is not None else None
            stack.callback(lambda: setattr(self, "training_iterator", None))
            if self.latest_checkpoint is not None:
                with self.core_context.checkpoint.restore_path(self.latest_checkpoint) as load_path:
                    self._load(load_path)
            else:
                self.state = _TrialState(trial_id=self.trial_id)
            for cb in self.callbacks.values():
                cb.on_training_start()
            with _grad.step_stream(self.context.device), self._profiling():
                self._run()

    # ------------------------------------------------------------------ DeepSpeed autotune mode
    def _run(self) -> None:
        try:
            hp = self.context.get_hparams()
        except ValueError:
            hp = {}
        if hp.get(dsat_defaults.USE_DSAT_MODE_KEY):
            return self._run_dsat(hp)
        return super()._run()

    def _run_dsat(self, hp: Dict[str, Any]) -> None:
        """Profiling trial of a dsat search (reference: `_deepspeed_trial.py` _dsat_mode +
        `dsat/_utils.py` dsat_reporting_context): train ``end`` batches, time batches
        [start, end), report throughput/latency(/FLOPS) as validation metrics and complete the
        searcher operation with the configured metric. An OOM ends the trial as InvalidHP."""
        start, end = (hp.get(dsat_defaults.PROFILE_KEY) or [3, 5])[:2]
        ctx = self.context
        if self.local_training:
            ops: Iterator[Any] = iter([core.DummySearcherOperation(end, self.is_chief)])
        else:
            ops = self.core_context.searcher.operations()
        op = next(iter(ops))
        calls = 1 if (ctx.use_pipeline_parallel or ctx._manual_grad_accumulation) else ctx.num_micro_batches_per_slot
        for m in ctx.models:
            m.train()

        def sync() -> float:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            ctx.distributed.allgather(None)
            return time.perf_counter()

        t0 = t1 = 0.0
        try:
            for step in range(end):
                if step == start:
                    t0 = sync()
                for _ in range(calls):
                    self.trial.train_batch(self.training_iterator, 0, step)
                self.state.batches_trained += 1
            t1 = sync()
        except SystemExit:
            # the engine's autotuning hook (config "autotuning" section, pytorch/deepspeed/
            # _autotune.py) measured the run -- a model profile or the profiled steps -- and wrote
            # its json: report that instead of this loop's own timing
            found = [p for p in (dsat_defaults.MODEL_INFO_PROFILING_PATH,
                                 dsat_defaults.AUTOTUNING_RESULTS_PATH) if os.path.exists(p)]
            if len(found) != 1:
                raise
            with open(found[0]) as f:
                res = json.load(f)
            if self.is_chief:
                self.core_context.train.report_validation_metrics(max(1, self.state.batches_trained), res)
                op.report_progress(end)
                op.report_completed(res)
            for _ in ops:
                pass
            return
        except torch.cuda.OutOfMemoryError as e:
            raise errors.InvalidHP(f"out of memory at micro batch {ctx.train_micro_batch_size_per_gpu}") from e
        except RuntimeError as e:
            if "out of memory" in str(e).lower():
                raise errors.InvalidHP(str(e)) from e
            raise
        n = max(1, end - start)
        dt = max(t1 - t0, 1e-9)
        samples = ctx.train_micro_batch_size_per_gpu * ctx.num_micro_batches_per_slot * ctx.distributed.size * n
        metrics = {"throughput": samples / dt, "latency": dt / n * 1000.0}
        module = getattr(ctx.models[0], "module", ctx.models[0])
        if hasattr(module, "flops_per_token") and hasattr(module, "cfg"):
            tokens = samples * module.cfg.max_seq_len
            metrics["FLOPS_per_gpu"] = tokens * module.flops_per_token() / dt / ctx.distributed.size
        if self.is_chief:
            self.core_context.train.report_validation_metrics(self.state.batches_trained, metrics)
            name = self.searcher_metric_name if self.searcher_metric_name in metrics else "throughput"
            op.report_progress(end)
            op.report_completed(metrics[name])
        for _ in ops:  # drain: the search method closes the trial
            pass

    # ------------------------------------------------------------------ training
    def _train_with_boundaries(self, boundaries):
        ctx = self.context
        metrics: List[Dict[str, Any]] = []
        if self.is_chief:
            self.core_context.train.set_status("training")
        self.prof.set_training(True)
        for m in ctx.models:
            m.train()
        ctx.reset_reducers()
        epoch_len = ctx._epoch_len
        calls = 1 if (ctx.use_pipeline_parallel or ctx._manual_grad_accumulation) else \
            ctx.num_micro_batches_per_slot
        while True:
            batch_idx = self.state.batches_trained
            epoch_idx, in_epoch = divmod(batch_idx, epoch_len)
            ctx._current_batch_idx = batch_idx
            if in_epoch == 0:
                for cb in self.callbacks.values():
                    cb.on_training_epoch_start(epoch_idx)
            ctx._loss_ids = {}
            self.prof.update_batch_idx(batch_idx)
            t0 = time.time()
            for _ in range(calls):
                # the torch profiler (set_profiler) was entered once around the loop (_profiling)
                with self.prof.record_timing("train_batch", requires_sync=False, accumulate=True):
                    out = self.trial.train_batch(self.training_iterator, epoch_idx, batch_idx)
                if ctx.profiler:
                    ctx.profiler.step()
                if ctx._mpu.should_report_metrics:
                    if isinstance(out, torch.Tensor):
                        out = {"loss": out}
                    if not isinstance(out, dict):
                        raise errors.InvalidExperimentException(
                            "train_batch must return a dictionary mapping string names to Tensor "
                            f"metrics, got {type(out)}")
                    metrics.append({k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()})
            m0 = ctx.models[0]
            if isinstance(m0, DeepSpeedEngine) and not ctx._manual_grad_accumulation and \
                    m0.micro_steps % ctx.num_micro_batches_per_slot != 0:
                raise RuntimeError("did not train for gradient accumulation steps")
            dt = time.time() - t0
            if dt > 0:
                self.prof.record_metric("samples_per_second",
                                        ctx.train_micro_batch_size_per_gpu * ctx.num_micro_batches_per_slot
                                        * ctx.distributed.size / dt)
            self._step_batch()
            for b in boundaries:
                if isinstance(b.unit, Batch) and b.unit.should_stop(batch_idx + 1):
                    b.limit_reached = True
                if not isinstance(b.unit, Batch) and b.unit.should_stop(epoch_idx + 1) and in_epoch == epoch_len - 1:
                    b.limit_reached = True
                if b.step_type == "TRAIN" and self.test_mode:
                    b.limit_reached = True
            if any(b.limit_reached for b in boundaries):
                return boundaries, metrics

    # ------------------------------------------------------------------ validation
    def _compute_validation_metrics(self) -> Dict[str, Any]:
        ctx = self.context
        for cb in self.callbacks.values():
            cb.on_validation_epoch_start()
        it = iter(self.validation_loader) if self.validation_loader is not None else None
        keys = None
        batch_metrics: List[Dict[str, Any]] = []
        for idx in range(int(self.num_validation_batches or 0)):
            vm = self.trial.evaluate_batch(it, idx)
            if ctx._mpu.should_report_metrics:
                if not isinstance(vm, dict):
                    raise errors.InvalidExperimentException(
                        "evaluate_batch must return a dictionary of string names to Tensor metrics")
                if keys is None:
                    keys = vm.keys()
                elif keys != vm.keys():
                    raise errors.InvalidExperimentException(
                        "Validation metric names must match across all batches of data.")
                batch_metrics.append({k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in vm.items()})
            if self.test_mode:
                break
        all_keys = [list(k) for k in ctx.distributed.allgather(list(keys) if keys is not None else None) if k is not None]
        keys = all_keys[0] if all_keys else []
        for cb in self.callbacks.values():
            cb.on_validation_epoch_end(batch_metrics)
        return _reducer.reduce_validation_metrics(
            ctx.distributed, batch_metrics, keys,
            _reducer._prepare_metrics_reducers(self.trial.evaluation_reducer(), keys=keys))

    # ------------------------------------------------------------------ checkpoint
    def _save(self, path: pathlib.Path) -> None:
        path.mkdir(parents=True, exist_ok=True)
        ctx = self.context
        rank = ctx.distributed.rank
        if self.is_chief:
            util.write_user_code(path, not self.local_training)
            (path / "trial_state.json").write_text(json.dumps(vars(self.state)))
            try:
                exp_conf, hparams = ctx.get_experiment_config(), ctx.get_hparams()
            except ValueError:
                exp_conf, hparams = None, None
            tc = type(self.trial)
            (path / "load_data.json").write_text(json.dumps(
                {"trial_type": "DeepSpeedTrial", "experiment_config": exp_conf, "hparams": hparams,
                 "trial_cls_spec": f"{tc.__module__}:{tc.__qualname__}"}, default=str))
        ckpt = {"rng_state": _rng_state(ctx.distributed.local_rank),
                "callbacks": {n: cb.state_dict() for n, cb in self.callbacks.items()}}
        for cb in self.callbacks.values():
            cb.on_checkpoint_save_start(ckpt)
        torch.save(ckpt, str(path / f"det_state_dict_rank{rank}.pth"))
        self.trial.save(ctx, path)
        for cb in self.callbacks.values():
            cb.on_checkpoint_end(str(path))
            cb.on_checkpoint_write_end(str(path))

    def _load(self, load_path: pathlib.Path) -> None:
        ctx = self.context
        p = load_path / f"det_state_dict_rank{ctx.distributed.rank}.pth"
        if not p.exists():
            self.state = _TrialState(trial_id=self.trial_id)
            return
        ckpt = load_state_dict_file(str(p))
        for cb in self.callbacks.values():
            cb.on_checkpoint_load_start(ckpt)
        self.trial.load(ctx, load_path)
        if "rng_state" in ckpt:
            _set_rng_state(ckpt["rng_state"], ctx.distributed.local_rank)
        for name, cb in self.callbacks.items():
            if name in ckpt.get("callbacks", {}):
                cb.load_state_dict(ckpt["callbacks"][name])
        st_path = load_path / "trial_state.json"
        if st_path.exists():
            st = json.loads(st_path.read_text())
            self.state = _TrialState(**st) if st.get("trial_id") == self.trial_id else _TrialState(trial_id=self.trial_id)
        else:
            self.state = _TrialState(trial_id=self.trial_id)


# ---------------------------------------------------------------------------------- entry points
@contextlib.contextmanager
def init(*, hparams: Optional[Dict] = None, exp_conf: Optional[Dict[str, Any]] = None,
         distributed: Optional[core.DistributedContext] = None) -> Iterator[DeepSpeedTrialContext]:
    """Build a :class:`DeepSpeedTrialContext` (on-cluster from DET_CLUSTER_INFO, else local)."""
    from determined_clone_amd.pytorch import _trainer

    info = _info.get_cluster_info()
    local = info is None or info.task_type != "TRIAL"
    dist_ctx = distributed
    if local:
        seed, steps_completed = None, 0
        num_gpus = torch.cuda.device_count() if torch.cuda.is_available() else 0
        if dist_ctx is None:
            dist_ctx = _trainer._initialize_distributed_backend()
    else:
        dist_ctx = dist_ctx or _trainer._initialize_distributed_backend()
        seed = info.trial.trial_seed
        exp_conf = info.trial._config
        hparams = hparams if hparams is not None else info.trial.hparams
        steps_completed = info.trial._steps_completed
        num_gpus = len(info.gpu_uuids) or (torch.cuda.device_count() if torch.cuda.is_available() else 0)
        _trainer._set_random_seeds(seed)
    with core.init(distributed=dist_ctx, preempt_mode=core.PreemptMode.WorkersAskChief,
                   tensorboard_mode=core.TensorboardMode.MANUAL) as core_context:
        yield DeepSpeedTrialContext(core_context=core_context, trial_seed=seed, hparams=hparams,
                                    slots_per_trial=core_context.distributed.get_size(),
                                    num_gpus=num_gpus, exp_conf=exp_conf, aggregation_frequency=1,
                                    steps_completed=steps_completed)


class Trainer:
    """``fit()`` for DeepSpeedTrials (same arguments as :class:`pytorch.Trainer.fit`)."""

    def __init__(self, trial: DeepSpeedTrial, context: DeepSpeedTrialContext) -> None:
        self._trial = trial
        self._context = context
        self._info = _info.get_cluster_info()
        self._local = self._info is None or self._info.task_type != "TRIAL"

    def fit(self, checkpoint_period: Optional[TrainUnit] = None,
            validation_period: Optional[TrainUnit] = None, max_length: Optional[TrainUnit] = None,
            reporting_period: TrainUnit = Batch(100),  # noqa: B008
            checkpoint_policy: str = "best", latest_checkpoint: Optional[str] = None,
            step_zero_validation: bool = False, test_mode: bool = False) -> DeepSpeedTrialController:
        if self._local:
            if max_length is None:
                raise ValueError("max_length must be defined in local training mode.")
            if checkpoint_policy == "best":
                checkpoint_policy = "all"
            smaller, metric, steps, gbs = True, None, 0, None
        else:
            cfg = self._info.trial._config
            smaller = bool(cfg["searcher"]["smaller_is_better"])
            metric = cfg["searcher"]["metric"]
            steps = int(self._info.trial._steps_completed)
            gbs = self._context.models[0].train_batch_size() if self._context.models else None
        c = DeepSpeedTrialController(
            trial_inst=self._trial, context=self._context,
            checkpoint_period=checkpoint_period or Batch(sys.maxsize),
            validation_period=validation_period or Batch(sys.maxsize),
            reporting_period=reporting_period, smaller_is_better=smaller, steps_completed=steps,
            latest_checkpoint=latest_checkpoint, local_training=self._local, test_mode=test_mode,
            searcher_metric_name=metric, checkpoint_policy=checkpoint_policy,
            step_zero_validation=step_zero_validation, max_length=max_length, global_batch_size=gbs)
        c.run()
        return c


def run_deepspeed_trial(trial_cls: type, info: Any) -> int:
    """Harness entry for ``entrypoint: module:DeepSpeedTrialSubclass`` experiments."""
    from determined_clone_amd.exec.harness import _unit

    cfg = info.trial._config
    with init() as ctx:
        trial = trial_cls(ctx)
        gbs = ctx.models[0].train_batch_size() if ctx.models else None
        rpe = int(cfg.get("records_per_epoch") or 0)
        Trainer(trial, ctx).fit(
            checkpoint_period=_unit(cfg["min_checkpoint_period"], gbs, rpe),
            validation_period=_unit(cfg["min_validation_period"], gbs, rpe),
            reporting_period=Batch(int(cfg.get("scheduling_unit") or 100)),
            checkpoint_policy=cfg.get("checkpoint_policy", "best"),
            latest_checkpoint=info.latest_checkpoint,
            step_zero_validation=bool(cfg.get("perform_initial_validation")))
    return 0
