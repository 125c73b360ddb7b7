"""PyTorchTrialContext (reference: `harness/determined/pytorch/_pytorch_context.py`).

Same user-facing API (wrap_model / wrap_optimizer / wrap_lr_scheduler / wrap_scaler / backward /
step_optimizer / to_device / hparams ...) on an MI355X engine:

* every wrapped optimizer's parameters are laid out in flat per-dtype buffers
  (`parallel/flat.py`); ``torch.optim.SGD/Adam/AdamW`` are swapped for the fused HIP optimizers
  (`ops/optim.py`) unless ``fused=False``;
* data-parallel gradient sync is bucketed in-place RCCL all-reduce overlapped with backward
  (`parallel/ddp.py`) instead of Horovod / torch DDP; averaging across ranks and over
  ``aggregation_frequency`` is folded into the fused optimizer's gradient multiplier;
* gradient clipping via :func:`clip_grad_norm` runs on-device inside the optimizer step (no
  host sync), AMP loss scaling uses the device-resident scaler.
"""
import contextlib
import logging
import pathlib
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Set, Tuple, Union

import torch

from determined_clone_amd import errors
from determined_clone_amd.ops import _grad
from determined_clone_amd.ops import optim as fused_optim
from determined_clone_amd.parallel import ddp
from determined_clone_amd.parallel.flat import FlatParamSpace
from determined_clone_amd.pytorch import _data
from determined_clone_amd.pytorch._lr_scheduler import LRScheduler
from determined_clone_amd.pytorch._reducer import _PyTorchReducerContext

logger = logging.getLogger("determined_clone_amd.pytorch")


class ClipGradNorm:
    """Marker clip function recognised by ``step_optimizer``: with a fused optimizer the global
    L2 norm + scaling run on the device inside the optimizer step; otherwise it falls back to
    ``torch.nn.utils.clip_grad_norm_``."""

    def __init__(self, max_norm: float) -> None:
        self.max_norm = float(max_norm)

    def __call__(self, params: Any) -> Any:
        return torch.nn.utils.clip_grad_norm_(list(params), self.max_norm)


def clip_grad_norm(max_norm: float) -> ClipGradNorm:
    return ClipGradNorm(max_norm)


class _Experimental:
    def __init__(self, ctx: "PyTorchTrialContext") -> None:
        self._ctx = ctx
        self._auto_amp = False
        self._auto_to_device = True
        self._data_repro_checks = True
        self.amp_dtype = torch.float16

    def use_amp(self, dtype: torch.dtype = torch.float16) -> None:
        """Automatic mixed precision: autocast the wrapped models' forward and (for fp16) scale the
        loss with a device-resident dynamic loss scaler."""
        self._auto_amp = True
        self.amp_dtype = dtype
        if dtype == torch.float16 and self._ctx._scaler is None:
            self._ctx.wrap_scaler(fused_optim.DeviceGradScaler(device=self._ctx.device))
        for i, m in enumerate(self._ctx.models):
            self._ctx.models[i] = self._ctx.autocast_forward_pass(m)

    def use_hip_graph(self, warmup_steps: int = 3) -> None:
        """Capture ``train_batch`` as a HIP graph after ``warmup_steps`` eager steps and replay it
        (same as ``optimizations.hip_graph: true``; see ``pytorch/_graph.py`` for requirements)."""
        self._ctx._hip_graph = True
        self._ctx._hip_graph_warmup = int(warmup_steps)

    def disable_auto_to_device(self) -> None:
        self._auto_to_device = False

    def disable_dataset_reproducibility_checks(self) -> None:
        self._data_repro_checks = False


class PyTorchTrialContext(_PyTorchReducerContext):
    def __init__(self, core_context: Any, trial_seed: Optional[int], hparams: Optional[Dict],
                 slots_per_trial: int, num_gpus: int, exp_conf: Optional[Dict[str, Any]],
                 aggregation_frequency: int = 1, steps_completed: int = 0,
                 managed_training: bool = True, debug_enabled: bool = False,
                 enable_tensorboard_logging: bool = True) -> None:
        self._core = core_context
        self.distributed = core_context.distributed
        super().__init__(self.distributed.allgather)
        self._per_slot_batch_size, self._global_batch_size = None, None
        self._hparams = hparams
        self._trial_seed = trial_seed
        self._slots_per_trial = slots_per_trial
        self._num_gpus = num_gpus
        self._exp_conf = exp_conf
        self._aggregation_frequency = aggregation_frequency
        self._steps_completed = steps_completed
        self._managed_training = managed_training
        self._debug_enabled = debug_enabled
        self._enable_tensorboard_logging = enable_tensorboard_logging
        opts = (exp_conf or {}).get("optimizations", {}) or {}
        self._average_aggregated_gradients = bool(opts.get("average_aggregated_gradients", True))
        self._gradient_compression = bool(opts.get("gradient_compression", False))
        self._average_training_metrics = bool(opts.get("average_training_metrics", True))
        self._hip_graph = bool(opts.get("hip_graph", False))
        self._hip_graph_warmup = int(opts.get("hip_graph_warmup_steps", 3) or 3)
        self._hip_graph_det_convs = bool(opts.get("hip_graph_deterministic_convs", False))
        fusion_mb = opts.get("tensor_fusion_threshold")
        self._bucket_mb = float(fusion_mb) if fusion_mb and fusion_mb != 64 else 32.0

        self.device = self._init_device()
        self.models: List[torch.nn.Module] = []
        self.optimizers: List[torch.optim.Optimizer] = []
        self.lr_schedulers: List[LRScheduler] = []
        self._scaler: Any = None
        self._syncs: Dict[int, ddp.GradientSync] = {}  # id(optimizer) -> gradient sync
        # id(user optimizer) -> the fused optimizer wrap_optimizer replaced it with
        self._optimizer_alias: Dict[int, torch.optim.Optimizer] = {}
        self._spaces: Dict[int, FlatParamSpace] = {}
        self._loose_params: Dict[int, List[torch.Tensor]] = {}
        self._current_batch_idx: Optional[int] = None
        self._epoch_len: Optional[int] = None
        self._stop_requested = False
        self._is_pre_trainer = False
        self._loss_ids: Dict[Any, int] = {}
        self.profiler: Any = None
        self._timings: Dict[str, float] = {}
        self.experimental = _Experimental(self)
        self._tbd_writer: Any = None
        self._main_model: Optional[torch.nn.Module] = None
        self._broadcasted: Set[int] = set()

        if hparams is not None and "global_batch_size" in hparams:
            gbs = int(hparams["global_batch_size"])
            if gbs < slots_per_trial:
                raise errors.InvalidExperimentException(
                    f"global_batch_size ({gbs}) must be >= slots_per_trial ({slots_per_trial})")
            self._global_batch_size = gbs
            self._per_slot_batch_size = gbs // slots_per_trial
            if gbs % slots_per_trial:
                logger.warning(f"global_batch_size {gbs} not divisible by slots_per_trial "
                               f"{slots_per_trial}; effective global batch is "
                               f"{self._per_slot_batch_size * slots_per_trial}")

    # ------------------------------------------------------------------ config accessors
    def get_global_batch_size(self) -> int:
        if self._global_batch_size is None:
            raise ValueError("global_batch_size is not a hyperparameter of this trial")
        return self._global_batch_size

    def get_per_slot_batch_size(self) -> int:
        if self._per_slot_batch_size is None:
            raise ValueError("global_batch_size is not a hyperparameter of this trial")
        return self._per_slot_batch_size

    def get_experiment_config(self) -> Dict[str, Any]:
        if self._exp_conf is None:
            raise ValueError("no experiment config is available in this context")
        return self._exp_conf

    def get_hparam(self, name: str) -> Any:
        if self._hparams is None:
            raise ValueError("no hyperparameters were provided to this context")
        if name not in self._hparams:
            raise ValueError(f"'{name}' is not one of the configured hyperparameters "
                             f"{sorted(self._hparams)}")
        return self._hparams[name]

    def get_hparams(self) -> Dict[str, Any]:
        if self._hparams is None:
            raise ValueError("no hyperparameters were provided to this context")
        return self._hparams

    def get_data_config(self) -> Dict[str, Any]:
        return (self._exp_conf or {}).get("data", {}) or {}

    def get_stop_requested(self) -> bool:
        return self._stop_requested

    def set_stop_requested(self, stop_requested: bool) -> None:
        if not isinstance(stop_requested, bool):
            raise AssertionError("stop_requested must be a boolean")
        self._stop_requested = stop_requested

    def set_enable_tensorboard_logging(self, enable: bool) -> None:
        self._enable_tensorboard_logging = bool(enable)

    def get_enable_tensorboard_logging(self) -> bool:
        return self._enable_tensorboard_logging

    def get_trial_seed(self) -> int:
        return self._trial_seed or 0

    def get_initial_batch(self) -> int:
        return self._steps_completed

    def get_experiment_id(self) -> int:
        return self._core.train._exp_id if self._core.train is not None else 0

    def get_trial_id(self) -> int:
        return self._core.train._trial_id if self._core.train is not None else 0

    def get_tensorboard_path(self) -> pathlib.Path:
        return self._core.train.get_tensorboard_path()

    def get_tensorboard_writer(self) -> Any:
        if self._tbd_writer is None:
            from determined_clone_amd import tensorboard

            self._tbd_writer = tensorboard.EventFileWriter(str(self.get_tensorboard_path()))
        return self._tbd_writer

    # ------------------------------------------------------------------ device
    def _init_device(self) -> torch.device:
        if torch.cuda.is_available() and self._num_gpus > 0:
            dev = torch.device("cuda", self.distributed.local_rank % torch.cuda.device_count())
            torch.cuda.set_device(dev)
            return dev
        return torch.device("cpu")

    def to_device(self, data: Any) -> Any:
        return _data.to_device(data, self.device)

    # ------------------------------------------------------------------ wrapping
    def wrap_model(self, model: torch.nn.Module) -> torch.nn.Module:
        model = model.to(self.device)
        if self._main_model is None:
            self._main_model = model
        self.models.append(model)
        if self.distributed.size > 1:
            ddp.broadcast_module_state(model)
        return model

    def autocast_forward_pass(self, to_wrap: torch.nn.Module) -> torch.nn.Module:
        ctx = self
        orig_forward = to_wrap.forward

        def forward(*args: Any, **kwargs: Any) -> Any:
            with torch.autocast(device_type=ctx.device.type, dtype=ctx.experimental.amp_dtype):
                return orig_forward(*args, **kwargs)

        to_wrap.forward = forward  # type: ignore[assignment]
        return to_wrap

    def wrap_optimizer(self, optimizer: torch.optim.Optimizer, backward_passes_per_step: int = 1,
                       fused: Optional[bool] = None) -> torch.optim.Optimizer:
        """Register an optimizer. With ``fused`` (default on GPU) a torch SGD/Adam/AdamW is
        replaced by its flat-buffer HIP equivalent; use the RETURNED optimizer."""
        if fused is None:
            fused = self.device.type == "cuda"
        out: torch.optim.Optimizer = optimizer
        if fused:
            f = fused_optim.fuse_optimizer(optimizer)
            if f is not None:
                out = f
        if out is not optimizer:
            # the reference hands back the user's own optimizer object; code that keeps using the
            # original (step_optimizer(orig), LR schedulers built on it) must drive the fused
            # replacement: alias it for step_optimizer and share the param-group dicts so
            # hyper-parameter changes made through either object reach the one that trains
            self._optimizer_alias[id(optimizer)] = out
            optimizer.param_groups = out.param_groups
        if isinstance(out, fused_optim.FusedOptimizerBase):
            space = out.space
        else:
            space = FlatParamSpace([g["params"] for g in out.param_groups])
        self._spaces[id(out)] = space
        if self.distributed.size > 1:
            comm_dtype = torch.bfloat16 if self._gradient_compression else None
            sync = ddp.GradientSync(space, bucket_mb=self._bucket_mb, comm_dtype=comm_dtype,
                                    average=True)
            if isinstance(out, fused_optim.FusedOptimizerBase):
                sync.fold_average = True
            self._syncs[id(out)] = sync
        self._update_grad_multiplier(out)
        self.optimizers.append(out)
        return out

    def _update_grad_multiplier(self, opt: torch.optim.Optimizer) -> None:
        if not isinstance(opt, fused_optim.FusedOptimizerBase):
            return
        mult = 1.0
        if self.distributed.size > 1:
            mult /= self.distributed.size
        if self._average_aggregated_gradients and self._aggregation_frequency > 1:
            mult /= self._aggregation_frequency
        opt.grad_multiplier = mult

    def wrap_lr_scheduler(self, lr_scheduler: Any, step_mode: LRScheduler.StepMode,
                          frequency: int = 1) -> LRScheduler:
        w = LRScheduler(lr_scheduler, step_mode, frequency)
        self.lr_schedulers.append(w)
        return w

    def wrap_scaler(self, scaler: Any) -> Any:
        self._scaler = scaler
        return scaler

    def configure_apex_amp(self, models: Any, optimizers: Any, enabled: bool = True,
                           opt_level: str = "O1", **kwargs: Any) -> Tuple[Any, Any]:
        """apex is CUDA-only; emulated with native AMP: O1 = fp16 autocast + dynamic loss scale,
        O2/O3 = bf16 autocast (no scaler needed on MI355X)."""
        if enabled:
            self.experimental.use_amp(torch.float16 if opt_level in ("O1",) else torch.bfloat16)
        return models, optimizers

    def set_profiler(self, *args: Any, **kwargs: Any) -> None:
        self.profiler = torch.profiler.profile(*args, **kwargs)

    # ------------------------------------------------------------------ training step
    def _should_communicate_and_update(self) -> bool:
        if not self._managed_training:
            return True
        if self._current_batch_idx is None:
            raise errors.InternalException("Training hasn't started.")
        return (self._current_batch_idx + 1) % self._aggregation_frequency == 0

    @contextlib.contextmanager
    def _no_sync(self) -> Iterator[None]:
        with contextlib.ExitStack() as st:
            for s in self._syncs.values():
                st.enter_context(s.no_sync())
            yield

    @contextlib.contextmanager
    def _record_timing(self, name: str, accumulate: bool = False) -> Iterator[None]:
        t0 = time.time()
        yield
        dt = time.time() - t0
        self._timings[name] = self._timings.get(name, 0.0) + dt if accumulate else dt

    def backward(self, loss: torch.Tensor, gradient: Optional[torch.Tensor] = None,
                 retain_graph: bool = False, create_graph: bool = False) -> None:
        if self._scaler is not None and self.experimental._auto_amp:
            loss = self._scaler.scale(loss)
        if self.distributed.size > 1 and not self._should_communicate_and_update():
            with self._no_sync():
                loss.backward(gradient=gradient, retain_graph=retain_graph, create_graph=create_graph)
        else:
            loss.backward(gradient=gradient, retain_graph=retain_graph, create_graph=create_graph)
        if loss.is_cuda:
            _grad.join()  # side-stream weight gradients (ops/_grad.py) complete before any reader

    def step_optimizer(self, optimizer: torch.optim.Optimizer,
                       clip_grads: Optional[Callable[[Iterator], None]] = None,
                       auto_zero_grads: bool = True, scaler: Optional[Any] = None) -> None:
        if self._aggregation_frequency > 1 and not auto_zero_grads:
            raise errors.InvalidExperimentException(
                "if optimizations.aggregation_frequency is larger than 1, auto_zero_grads must be true")
        if not self._should_communicate_and_update():
            return
        if torch.cuda.is_available():
            _grad.join()  # loss.backward() called directly: side-stream gradients land first
        optimizer = self._optimizer_alias.get(id(optimizer), optimizer)
        if self.distributed.size > 1 and all(optimizer is not o for o in self.optimizers):
            # an unregistered optimizer would step on un-all-reduced gradients: ranks diverge
            raise errors.InvalidExperimentException(
                "step_optimizer() got an optimizer that was not passed through wrap_optimizer(); "
                "its gradients would not be synchronised across slots")
        sync = self._syncs.get(id(optimizer))
        if sync is not None:
            sync.finish()
        if scaler is None and self.experimental._auto_amp:
            scaler = self._scaler
        fused = isinstance(optimizer, fused_optim.FusedOptimizerBase)
        params = [p for g in optimizer.param_groups for p in g.get("params", [])]
        if not fused and self._average_aggregated_gradients and self._aggregation_frequency > 1:
            for p in params:
                if p.grad is not None:
                    p.grad.div_(self._aggregation_frequency)
        if fused:
            max_norm = clip_grads.max_norm if isinstance(clip_grads, ClipGradNorm) else 0.0
            if clip_grads is not None and not isinstance(clip_grads, ClipGradNorm):
                # arbitrary user clip fn: needs true (unscaled, averaged) grads in place
                if scaler is not None:
                    scaler.unscale_(optimizer) if isinstance(scaler, fused_optim.DeviceGradScaler) else None
                self._materialize_grad_scale(optimizer)
                clip_grads(params)
            if isinstance(scaler, fused_optim.DeviceGradScaler):
                scaler.step(optimizer, max_norm=max_norm)
            elif scaler is not None:
                optimizer.prepare_grads(max_norm=max_norm)
                scaler.step(optimizer)
            else:
                if max_norm > 0:
                    optimizer.prepare_grads(max_norm=max_norm)
                optimizer.step()
        else:
            if clip_grads is not None:
                if scaler is not None:
                    scaler.unscale_(optimizer)
                clip_grads(params)
            if scaler is not None:
                scaler.step(optimizer)
            else:
                optimizer.step()
        if auto_zero_grads:
            optimizer.zero_grad()

    def _materialize_grad_scale(self, optimizer: fused_optim.FusedOptimizerBase) -> None:
        """Apply the folded multiplier to the gradients themselves (needed before a user clip fn)."""
        if optimizer._dev_scale is None:
            optimizer.prepare_grads()
        for st in optimizer.flat.values():
            st.buf.grad.mul_(optimizer._dev_scale[0].to(st.buf.grad.dtype))
        optimizer._dev_scale = torch.tensor([1.0, float(optimizer._dev_scale[1]), 0.0],
                                            device=optimizer._dev_scale.device)

    def _sync_buffers(self) -> None:
        """Broadcast non-parameter buffers (BN running stats) from rank 0 before eval/save."""
        if self.distributed.size > 1:
            import torch.distributed as dist

            for m in self.models:
                bufs = [b for b in m.buffers()]
                if bufs:
                    ddp._broadcast_coalesced(bufs, None, 0)

    # ------------------------------------------------------------------ epoch helpers
    def is_epoch_start(self) -> bool:
        if self._current_batch_idx is None:
            raise errors.InternalException("Training hasn't started.")
        if self._epoch_len is None:
            raise errors.InternalException("Training DataLoader uninitialized.")
        return self._current_batch_idx % self._epoch_len == 0

    def is_epoch_end(self) -> bool:
        if self._current_batch_idx is None:
            raise errors.InternalException("Training hasn't started.")
        if self._epoch_len is None:
            raise errors.InternalException("Training DataLoader uninitialized.")
        return self._current_batch_idx % self._epoch_len == self._epoch_len - 1

    def current_train_epoch(self) -> int:
        if self._current_batch_idx is None or self._epoch_len is None:
            raise errors.InternalException("Training hasn't started.")
        return self._current_batch_idx // self._epoch_len

    def current_train_batch(self) -> int:
        if self._current_batch_idx is None:
            raise errors.InternalException("Training hasn't started.")
        return self._current_batch_idx

    def _set_is_pre_trainer(self) -> None:
        self._is_pre_trainer = True
