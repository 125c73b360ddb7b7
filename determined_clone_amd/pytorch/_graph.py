"""HIP-graph capture of the training step (``optimizations.hip_graph``).

A ResNet-50 step on MI355X launches ~700 kernels; a small CNN's step is almost all launch
overhead. After a few eager warm-up steps (MIOpen algorithm search, allocator warm-up, optimizer
state creation) the controller captures ONE call of ``trial.train_batch`` -- forward, backward,
fused optimizer step, gradient zeroing -- into a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph
on ROCm) and replays it for every later batch:

* the batch is copied into static input tensors before each replay (same shapes required; a batch
  of another shape runs eagerly);
* the fused optimizers read lr and the step-dependent terms (Adam bias corrections, SGD's
  first-step momentum init) from a device buffer refreshed before each replay
  (``FusedOptimizerBase.refresh_device_hparams``), so LR schedules keep working;
* returned metric tensors are cloned after the replay (the graph's outputs are overwritten by the
  next replay).

Requirements (checked by :func:`unsupported_reason`): one GPU per trial (RCCL collectives are not
captured), ``aggregation_frequency == 1``, every wrapped optimizer a graph-capturable fused
optimizer, and a ``train_batch`` without host synchronisation or data-dependent Python control
flow. Transformer trials (fused LayerNorm / attention / bias-GELU / cross-entropy, hipBLASLt
GEMMs, fused AdamW with device-side clipping) and ResNets replay bit-exactly.

MIOpen convolutions: the eager-vs-replay difference measured in earlier rounds
(profiles/round4_hip_graph_miopen_root_cause.txt) was not a capture bug -- MIOpen's default solver
for small strided 1x1 NHWC convolutions (ConvAsmImplicitGemmGTCDynamicFwdXdlopsNHWC, a split-K
kernel accumulating with atomics) is nondeterministic run to run (relative 4e-5 between two EAGER
calls), and the replay merely ran it with a different atomic order. With
``optimizations.hip_graph_deterministic_convs: true`` every call of the step function made by the
runner (warm-up, capture, eager fallbacks) runs MIOpen's deterministic solvers
(``torch.backends.cudnn.deterministic = True`` for the duration of the call only), and eager and
replay agree bit for bit. It is OFF by default: the deterministic solvers made the CIFAR ASHA
trial's step ~10x slower (79.6 s vs 8.1 s for 300 batches, tools/probe_cifar_graph.py,
profiles/round5_asha_hip_graph_attempt.txt) -- a price only bitwise reproducibility should pay.
The reference has no equivalent (its step is eager).
"""
import contextlib
import logging
from typing import Any, Callable, Iterator, List, Optional

import torch
from torch.utils import _pytree as pytree

from determined_clone_amd.ops import optim as fused_optim

logger = logging.getLogger("determined_clone_amd.pytorch")


def unsupported_reason(context: Any) -> Optional[str]:
    if context.device.type != "cuda":
        return "not on a GPU"
    if context.distributed.size > 1:
        return "multi-GPU trials synchronise gradients with RCCL collectives outside the graph"
    if context._aggregation_frequency != 1:
        return "aggregation_frequency > 1"
    if not context.optimizers:
        return "no optimizer wrapped"
    for opt in context.optimizers:
        if not isinstance(opt, fused_optim.FusedOptimizerBase) or not opt.graph_capturable:
            return f"optimizer {type(opt).__name__} is not graph-capturable"
    return None


def _has_convs(context: Any) -> bool:
    convs = (torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d, torch.nn.ConvTranspose2d)
    return any(isinstance(mod, convs) for m in context.models for mod in m.modules())


class GraphedTrainStep:
    def __init__(self, context: Any, fn: Callable[..., Any], warmup_steps: int = 3,
                 deterministic_convs: bool = False) -> None:
        self.context = context
        self.fn = fn
        self.warmup_steps = max(1, int(warmup_steps))
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_in: List[Any] = []
        self.in_spec: Any = None
        self.static_out: Any = None
        self.replays = 0
        for opt in context.optimizers:
            opt.enable_device_hparams()
        # deterministic_convs: MIOpen runs its deterministic solvers for every call of the step
        # function this object makes (warm-up, capture, eager fallbacks), so warm-up, capture and
        # replay run the same solvers; the process-wide flag is restored after each call, so
        # evaluation, other models and later trials in the process keep the fastest solvers.
        self._deterministic = (deterministic_convs and torch.backends.cudnn.enabled
                               and not torch.backends.cudnn.deterministic and _has_convs(context))
        if self._deterministic:
            logger.info("hip_graph: MIOpen runs deterministic convolution solvers inside the "
                        "graphed training step")

    @contextlib.contextmanager
    def _solvers(self) -> Iterator[None]:
        if not self._deterministic:
            yield
            return
        prev = torch.backends.cudnn.deterministic
        torch.backends.cudnn.deterministic = True
        try:
            yield
        finally:
            torch.backends.cudnn.deterministic = prev

    def _eager(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        with self._solvers():
            return self.fn(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)

    # ------------------------------------------------------------------ helpers
    def _matches(self, leaves: List[Any], spec: Any) -> bool:
        if spec != self.in_spec or len(leaves) != len(self.static_in):
            return False
        for a, b in zip(leaves, self.static_in):
            if isinstance(b, torch.Tensor):
                if not isinstance(a, torch.Tensor) or a.shape != b.shape or a.dtype != b.dtype \
                        or a.device != b.device:
                    return False
            elif a != b:
                return False
        return True

    def _load_inputs(self, leaves: List[Any]) -> None:
        for a, b in zip(leaves, self.static_in):
            if isinstance(b, torch.Tensor):
                b.copy_(a, non_blocking=True)

    @staticmethod
    def _clone_out(out: Any) -> Any:
        return pytree.tree_map(lambda t: t.clone() if isinstance(t, torch.Tensor) else t, out)

    # ------------------------------------------------------------------ entry
    def __call__(self, batch: Any, epoch_idx: int, batch_idx: int) -> Any:
        self.calls += 1
        leaves, spec = pytree.tree_flatten(batch)
        if self.graph is None and self.calls <= self.warmup_steps:
            return self._eager(batch, epoch_idx, batch_idx)
        if self.graph is None:
            return self._capture(leaves, spec, epoch_idx, batch_idx)
        if not self._matches(leaves, spec):
            logger.debug("batch structure/shape differs from the captured one: running eagerly")
            return self._eager(batch, epoch_idx, batch_idx)
        self._load_inputs(leaves)
        for opt in self.context.optimizers:
            opt._step += 1  # the Python side of step() does not run on replay
            opt.refresh_device_hparams()
        self.graph.replay()
        self.replays += 1
        return self._clone_out(self.static_out)

    def _capture(self, leaves: List[Any], spec: Any, epoch_idx: int, batch_idx: int) -> Any:
        self.in_spec = spec
        self.static_in = [x.clone() if isinstance(x, torch.Tensor) else x for x in leaves]
        static_batch = pytree.tree_unflatten(self.static_in, spec)
        for opt in self.context.optimizers:
            opt.refresh_device_hparams(opt._step + 1)  # the step about to be captured
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g), self._solvers():
            self.static_out = self.fn(batch=static_batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
        self.graph = g
        logger.info("captured the training step as a HIP graph")
        g.replay()  # capture records without executing: run the captured step now
        self.replays += 1
        return self._clone_out(self.static_out)
