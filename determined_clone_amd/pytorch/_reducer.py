"""Metric reducers (reference: `harness/determined/pytorch/_reducer.py`, `_metric_utils.py`).

Difference from the reference: per-batch TRAINING metrics stay on the GPU until a reporting
boundary (the reference calls ``.cpu()`` on every batch, i.e. one device sync per step); at the
boundary they are stacked and averaged across ranks with ONE collective, then copied once.
"""
import abc
import enum
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np
import torch


class Reducer(enum.Enum):
    AVG = 1
    SUM = 2
    MAX = 3
    MIN = 4


def _simple_reduce_metrics(reducer: Reducer, metrics: np.ndarray,
                           num_batches: Optional[List[int]] = None) -> np.float64:
    if reducer == Reducer.AVG:
        if num_batches and len(metrics) != len(num_batches):
            raise RuntimeError(f"Lengths of metrics and num_batches are not equal: "
                               f"{len(metrics)} != {len(num_batches)}.")
        return np.average(metrics, weights=num_batches, axis=0)
    if reducer == Reducer.SUM:
        return np.sum(metrics, axis=0)
    if reducer == Reducer.MAX:
        return np.max(metrics, axis=0)
    if reducer == Reducer.MIN:
        return np.min(metrics, axis=0)
    raise NotImplementedError(reducer)


class MetricReducer(metaclass=abc.ABCMeta):
    """Custom reducer: ``update()`` per batch (user-called), ``per_slot_reduce()`` on each rank,
    ``cross_slot_reduce(per_slot_metrics)`` on the chief."""

    @abc.abstractmethod
    def reset(self) -> None:
        pass

    @abc.abstractmethod
    def per_slot_reduce(self) -> Any:
        pass

    @abc.abstractmethod
    def cross_slot_reduce(self, per_slot_metrics: List) -> Any:
        pass


class _SimpleReducer(MetricReducer):
    def __init__(self, fn: Callable) -> None:
        self.fn = fn
        self.reset()

    def reset(self) -> None:
        self.updates: List[Any] = []

    def update(self, value: Any) -> None:
        if isinstance(value, torch.Tensor):
            value = value.detach().cpu().numpy()
        self.updates.append(value)

    def per_slot_reduce(self) -> Any:
        return self.updates

    def cross_slot_reduce(self, per_slot_metrics: List) -> Any:
        flat = [x for slot in per_slot_metrics for x in slot]
        return self.fn(flat)


class _WrappedReducer:
    def __init__(self, reducer: MetricReducer, name: Optional[str], for_training: bool,
                 for_validation: bool) -> None:
        self.reducer = reducer
        self.name = name
        self.for_training = for_training
        self.for_validation = for_validation

    def reset(self) -> None:
        self.reducer.reset()

    def per_slot_reduce(self) -> Any:
        return self.reducer.per_slot_reduce()

    def cross_slot_reduce(self, per_slot_metrics: List) -> Any:
        return self.reducer.cross_slot_reduce(per_slot_metrics)


class _PyTorchReducerContext:
    def __init__(self, allgather_fn: Callable[[Any], List[Any]] = lambda x: [x]) -> None:
        self._wrapped_reducers: List[_WrappedReducer] = []
        self._allgather_fn = allgather_fn

    def reset_reducers(self) -> None:
        for w in self._wrapped_reducers:
            w.reset()

    def wrap_reducer(self, reducer: Union[Callable, MetricReducer], name: Optional[str] = None,
                     for_training: bool = True, for_validation: bool = True) -> Any:
        if isinstance(reducer, MetricReducer):
            wrapped = _WrappedReducer(reducer, name, for_training, for_validation)
        elif callable(reducer):
            reducer = _SimpleReducer(reducer)
            wrapped = _WrappedReducer(reducer, name, for_training, for_validation)
        else:
            raise TypeError("reducer must be a callable or a MetricReducer")
        if name is not None and any(w.name == name for w in self._wrapped_reducers):
            raise ValueError(f"a reducer named {name} is already registered")
        self._wrapped_reducers.append(wrapped)
        return reducer

    def run_cross_slot_reduction(self, reducables: List[_WrappedReducer], gathered: List[Any]) -> Dict[str, Any]:
        metrics: Dict[str, Any] = {}
        for wrapped, per_slot in zip(reducables, zip(*gathered)):
            reduced = wrapped.cross_slot_reduce(list(per_slot))
            if wrapped.name is None:
                if not isinstance(reduced, dict):
                    raise AssertionError("a reducer wrapped with name=None must return a dict of metrics")
                metrics.update(reduced)
            else:
                if isinstance(reduced, dict):
                    raise AssertionError(f"reducer '{wrapped.name}' was given a name but returned a dict")
                metrics[wrapped.name] = reduced
        return metrics

    def reduce_metrics(self, for_training: bool) -> Dict[str, Any]:
        reducables = [w for w in self._wrapped_reducers
                      if (for_training and w.for_training) or (not for_training and w.for_validation)]
        if not reducables:
            return {}
        gathered = self._allgather_fn([w.per_slot_reduce() for w in reducables])
        return self.run_cross_slot_reduction(reducables, gathered)


def _prepare_metrics_reducers(reducer: Union[Reducer, Dict[str, Reducer]], keys: Any) -> Dict[str, Reducer]:
    from determined_clone_amd.errors import InvalidExperimentException

    if isinstance(reducer, dict):
        if set(keys) != set(reducer.keys()):
            raise InvalidExperimentException(
                "provide a single evaluation reducer or one for every validation metric; "
                f"expected keys {sorted(keys)}, got {sorted(reducer.keys())}")
        out = dict(reducer)
    else:
        out = {k: reducer for k in keys}
    for k in keys:
        if not isinstance(out[k], Reducer):
            raise InvalidExperimentException("use determined_clone_amd.pytorch.Reducer for validation metrics")
    return out


def _to_numpy(v: Any) -> Any:
    if isinstance(v, torch.Tensor):
        return v.detach().float().cpu().numpy() if v.is_floating_point() else v.detach().cpu().numpy()
    return v


def reduce_validation_metrics(dist: Any, batch_metrics: List[Dict[str, Any]], keys: Any,
                              reducers: Dict[str, Reducer]) -> Dict[str, Any]:
    """Per-rank reduction of per-batch metrics, then batch-count-weighted cross-rank reduction on
    the chief (reference `_metric_utils._reduce_metrics`)."""
    metrics: Dict[str, Any] = {}
    if batch_metrics:
        metrics = {n: _simple_reduce_metrics(reducers[n], np.stack([_to_numpy(b[n]) for b in batch_metrics], 0))
                   for n in keys or []}
    if dist.size > 1:
        allv = dist.gather((metrics, len(batch_metrics)))
        if dist.rank != 0:
            return {}
        allv = [a for a in allv if a[1]]
        per_key = {n: np.stack([a[0][n] for a in allv], 0) for n in keys or []}
        nb = [a[1] for a in allv]
        metrics = {n: _simple_reduce_metrics(reducers[n], per_key[n], nb) for n in keys or []}
    return metrics


def average_training_metrics(dist: Any, batch_metrics: List[Dict[str, Any]],
                             average_across_ranks: bool) -> Dict[str, Any]:
    """Returns {"avg_metrics": ..., "batch_metrics": [...]} on the chief (others: same structure).

    Scalar tensor metrics are stacked on device as [num_batches, num_metrics]; if requested the
    stack is averaged across ranks with one all-reduce; then ONE device->host copy."""
    if not batch_metrics:
        return {"avg_metrics": {}, "batch_metrics": []}
    keys = list(batch_metrics[0].keys())
    tensor_keys = [k for k in keys if isinstance(batch_metrics[0][k], torch.Tensor)
                   and batch_metrics[0][k].numel() == 1]
    other_keys = [k for k in keys if k not in tensor_keys]
    per_batch: List[Dict[str, Any]] = [dict() for _ in batch_metrics]
    if tensor_keys:
        stack = torch.stack([torch.stack([b[k].detach().reshape(()).float() for k in tensor_keys])
                             for b in batch_metrics])
        if average_across_ranks and dist.size > 1:
            import torch.distributed as tdist

            if tdist.get_backend() == "gloo" and stack.is_cuda:
                cpu = stack.cpu()
                tdist.all_reduce(cpu)
                stack = cpu
            else:
                tdist.all_reduce(stack)
            stack = stack / dist.size
        host = stack.cpu().numpy()
        for i in range(len(batch_metrics)):
            for j, k in enumerate(tensor_keys):
                per_batch[i][k] = float(host[i, j])
    for k in other_keys:
        vals = [_to_numpy(b[k]) for b in batch_metrics]
        if average_across_ranks and dist.size > 1:
            allv = dist.allgather(vals)
            vals = [np.mean([np.asarray(r[i], dtype=np.float64) for r in allv], axis=0) for i in range(len(vals))]
        for i, v in enumerate(vals):
            per_batch[i][k] = v
    avg: Dict[str, Any] = {}
    for k in keys:
        col = [pb[k] for pb in per_batch if pb[k] is not None]
        try:
            avg[k] = float(np.mean(np.asarray(col, dtype=np.float64))) if col else None
        except (TypeError, ValueError):
            avg[k] = col[-1] if col else None
    return {"avg_metrics": avg, "batch_metrics": per_batch}
