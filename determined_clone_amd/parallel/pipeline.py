"""Pipeline parallelism: layer-spec models partitioned over stages, 1F1B schedule over P2P.

The reference's DeepSpeedTrial accepts a ``deepspeed.PipelineEngine`` (reference:
`harness/determined/pytorch/deepspeed/_deepspeed_context.py:188` sets ``use_pipeline_parallel``
and takes the data-parallel coordinates from the engine's grid, `_mpu.py:33`
``make_deepspeed_mpu``; `_deepspeed_trial.py:155` validation in units of
gradient-accumulation-steps micro-batches; `examples/deepspeed/gpt_neox/zero1.yaml:15`
``pipe_parallel_size: 2``). This module is the MI355X-native equivalent, built on
``torch.distributed`` point-to-point ops (RCCL over xGMI on the GPU box, gloo on CPU):

* :class:`LayerSpec` / :class:`TiedLayerSpec` describe layers lazily; :class:`PipelineModule`
  partitions them into ``num_stages`` contiguous stages (``"parameters"``: balanced by parameter
  count, counted on the ``meta`` device so no rank materialises the whole model;
  ``"uniform"``; ``"type:<regex>"``) and instantiates only the local stage.
* :class:`PipelineGrid`: ``rank = stage * dp + data_rank`` -- a stage's data-parallel replicas are
  adjacent ranks (adjacent GPUs share the most xGMI links for the per-step gradient
  all-reduce, which moves far more bytes than the per-micro-batch activations between stages).
* :class:`PipelineEngine` (a :class:`~determined_clone_amd.pytorch.deepspeed.DeepSpeedEngine`)
  runs ``train_batch(data_iter)`` as the non-interleaved 1F1B ("PipeDream-flush") schedule:
  ``stages - stage - 1`` warm-up forwards, then alternating forward/backward with the
  activation send fused with the gradient receive (``batch_isend_irecv``), then cool-down
  backwards. At most ``stages`` micro-batches of activations are live per stage, so activation
  memory is bounded independently of ``gradient_accumulation_steps``.
* Gradients: accumulate over micro-batches in the fused optimizer's flat buffer; the data-parallel
  bucketed all-reduce / ZeRO reduce-scatter fires during the LAST micro-batch's backward
  (overlapped), tied weights (e.g. GPT input embedding / LM head on the first and last stage)
  are summed over their tie group, the clip norm is summed over the pipeline group with each
  tied weight counted once, then one fused optimizer step per stage.
* Checkpoints are per layer (``layer_XX-model_states.pt``), so they reload under a different
  stage count; optimizer state reloads when the partition is unchanged.

Limitations (explicit errors): fp16 dynamic loss scaling (use bf16, the MI355X-native format),
activations must keep their shapes across the micro-batches of one ``train_batch`` call.
"""
import logging
import math
import pathlib
import re
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
from torch import nn

logger = logging.getLogger("determined_clone_amd.parallel.pipeline")

Activation = Union[torch.Tensor, Tuple[torch.Tensor, ...]]


# ---------------------------------------------------------------------------------- layer specs
class LayerSpec:
    """Lazily built layer: ``LayerSpec(nn.Linear, 16, 32)`` -> ``nn.Linear(16, 32)`` on the
    owning stage only."""

    def __init__(self, typename: type, *module_args: Any, **module_kwargs: Any) -> None:
        if not issubclass(typename, nn.Module):
            raise TypeError("LayerSpec only supports torch.nn.Module types")
        self.typename = typename
        self.module_args = module_args
        self.module_kwargs = module_kwargs

    def build(self) -> nn.Module:
        return self.typename(*self.module_args, **self.module_kwargs)

    def __repr__(self) -> str:
        return f"LayerSpec({self.typename.__name__})"


class TiedLayerSpec(LayerSpec):
    """A layer whose ``tied_weight_attr`` parameters are shared by every spec with the same
    ``key`` (on any stage). ``forward_fn(module, x)`` replaces ``module(x)`` when given, e.g. the
    LM head reusing the embedding table: ``forward_fn=lambda m, h: F.linear(h, m.wte.weight)``."""

    def __init__(self, key: str, typename: type, *module_args: Any,
                 forward_fn: Optional[Callable[[nn.Module, Any], Any]] = None,
                 tied_weight_attr: Union[str, Sequence[str]] = "weight", **module_kwargs: Any) -> None:
        super().__init__(typename, *module_args, **module_kwargs)
        self.key = key
        self.forward_fn = forward_fn
        self.tied_weight_attr = [tied_weight_attr] if isinstance(tied_weight_attr, str) \
            else list(tied_weight_attr)


def _get_attr(module: nn.Module, dotted: str) -> torch.Tensor:
    for part in dotted.split("."):
        module = getattr(module, part)
    return module  # type: ignore[return-value]


# ---------------------------------------------------------------------------------- partitioning
def partition_uniform(num_items: int, num_parts: int) -> List[int]:
    """Boundaries ``[0, ..., num_items]`` splitting items as evenly as possible."""
    if num_parts <= 0:
        raise ValueError("num_parts must be positive")
    base, extra = divmod(num_items, num_parts)
    parts = [0]
    for p in range(num_parts):
        parts.append(parts[-1] + base + (1 if p < extra else 0))
    return parts


def partition_balanced(weights: Sequence[float], num_parts: int) -> List[int]:
    """Contiguous partition of ``weights`` into ``num_parts`` non-empty parts minimising the
    heaviest part (exact dynamic program; layer lists are short)."""
    n, P = len(weights), num_parts
    if P >= n:
        return list(range(n + 1)) + [n] * (P - n)
    prefix = [0.0]
    for w in weights:
        prefix.append(prefix[-1] + float(w))
    inf = float("inf")
    best = [[inf] * (n + 1) for _ in range(P + 1)]
    cut = [[0] * (n + 1) for _ in range(P + 1)]
    best[0][0] = 0.0
    for k in range(1, P + 1):
        for i in range(k, n - (P - k) + 1):
            for j in range(k - 1, i):
                v = max(best[k - 1][j], prefix[i] - prefix[j])
                if v < best[k][i]:
                    best[k][i], cut[k][i] = v, j
    parts = [n]
    for k in range(P, 0, -1):
        parts.append(cut[k][parts[-1]])
    return parts[::-1]


def _count_params(spec: Any) -> int:
    if isinstance(spec, nn.Module):
        return sum(p.numel() for p in spec.parameters())
    if isinstance(spec, LayerSpec):
        with torch.device("meta"):
            return sum(p.numel() for p in spec.build().parameters())
    return 0


# ---------------------------------------------------------------------------------- topology
class PipelineGrid:
    """Stage x data-parallel process grid (DeepSpeed ``PipelineParallelGrid`` accessors, which
    ``make_deepspeed_mpu`` reads). Every rank must construct it (group creation is collective)."""

    def __init__(self, num_stages: int) -> None:
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0
        if num_stages <= 0 or self.world_size % num_stages:
            raise ValueError(f"world size {self.world_size} is not divisible by num_stages "
                             f"{num_stages}")
        self.pipe_parallel_size = num_stages
        self.data_parallel_size = self.world_size // num_stages
        self.stage_id, self.data_parallel_id = divmod(self.global_rank, self.data_parallel_size)
        self.pp_group: Any = None
        self.dp_group: Any = None
        self.pp_ranks = [self.stage_to_global(s) for s in range(num_stages)]
        self.dp_ranks = [self.stage_id * self.data_parallel_size + d
                         for d in range(self.data_parallel_size)]
        if dist.is_initialized() and self.world_size > 1:
            D, P = self.data_parallel_size, num_stages
            for d in range(D):
                ranks = [s * D + d for s in range(P)]
                g = dist.new_group(ranks)
                if self.global_rank in ranks:
                    self.pp_group = g
            if P == 1:
                self.dp_group = dist.group.WORLD
            else:
                for s in range(P):
                    ranks = [s * D + d for d in range(D)]
                    g = dist.new_group(ranks)
                    if self.global_rank in ranks:
                        self.dp_group = g

    model_parallel_size = 1  # no tensor parallelism (parallel.tensor.ModelParallelGrid has it)
    model_parallel_id = 0
    mp_group = None

    def stage_to_global(self, stage_id: int, data_parallel_id: Optional[int] = None,
                        model_parallel_id: Optional[int] = None) -> int:
        d = self.data_parallel_id if data_parallel_id is None else data_parallel_id
        return stage_id * self.data_parallel_size + d

    # DeepSpeed grid accessors
    def get_stage_id(self) -> int:
        return self.stage_id

    def get_pipe_parallel_rank(self) -> int:
        return self.stage_id

    def get_pipe_parallel_world_size(self) -> int:
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self) -> Any:
        return self.pp_group

    def get_data_parallel_rank(self) -> int:
        return self.data_parallel_id

    def get_data_parallel_world_size(self) -> int:
        return self.data_parallel_size

    def get_data_parallel_group(self) -> Any:
        return self.dp_group

    def get_slice_parallel_rank(self) -> int:
        return 0  # no tensor (slice) parallelism inside a stage

    def get_slice_parallel_world_size(self) -> int:
        return 1

    get_model_parallel_rank = get_slice_parallel_rank
    get_model_parallel_world_size = get_slice_parallel_world_size


# ---------------------------------------------------------------------------------- module
class PipelineModule(nn.Module):
    """Sequential model given as a list of :class:`LayerSpec` / modules / callables; holds only
    the local stage's layers. ``forward(x)`` runs the local stage; ``loss_fn(outputs, labels)``
    runs on the last stage."""

    def __init__(self, layers: Sequence[Any], num_stages: int = 1,
                 loss_fn: Optional[Callable[[Any, Any], torch.Tensor]] = None,
                 partition_method: str = "parameters", activation_checkpoint_interval: int = 0,
                 seed_layers: bool = False, base_seed: int = 1234,
                 grid: Optional[Any] = None) -> None:
        super().__init__()
        self.specs = list(layers)
        self.loss_fn = loss_fn
        self.activation_checkpoint_interval = int(activation_checkpoint_interval)
        self._grid = grid if grid is not None else PipelineGrid(num_stages)
        self.num_stages = self._grid.pipe_parallel_size
        self.stage_id = self._grid.stage_id
        self.parts = self._partition(partition_method)
        self._local_start, self._local_stop = self.parts[self.stage_id], self.parts[self.stage_id + 1]
        self.tied_modules = nn.ModuleDict()
        self.tied_weight_attrs: Dict[str, List[str]] = {}
        self.forward_funcs: List[Callable[[Any], Any]] = []
        self._layer_modules: Dict[int, nn.Module] = {}
        for idx in range(self._local_start, self._local_stop):
            spec = self.specs[idx]
            if seed_layers:
                torch.manual_seed(base_seed + idx)
            if isinstance(spec, TiedLayerSpec):
                if spec.key not in self.tied_modules:
                    self.tied_modules[spec.key] = spec.build()
                    self.tied_weight_attrs[spec.key] = spec.tied_weight_attr
                mod = self.tied_modules[spec.key]
                self._layer_modules[idx] = mod
                if spec.forward_fn is None:
                    self.forward_funcs.append(mod)
                else:
                    self.forward_funcs.append(lambda x, _f=spec.forward_fn, _m=mod: _f(_m, x))
            elif isinstance(spec, LayerSpec):
                mod = spec.build()
                self.add_module(str(idx), mod)
                self._layer_modules[idx] = mod
                self.forward_funcs.append(mod)
            elif isinstance(spec, nn.Module):
                self.add_module(str(idx), spec)
                self._layer_modules[idx] = spec
                self.forward_funcs.append(spec)
            elif callable(spec):
                self.forward_funcs.append(spec)
            else:
                raise TypeError(f"layer {idx}: unsupported pipeline layer {spec!r}")
        # key -> owning stages (every stage knows every tie, for the collective group setup)
        self.tie_stages: Dict[str, List[int]] = {}
        for idx, spec in enumerate(self.specs):
            if isinstance(spec, TiedLayerSpec):
                st = self._stage_of(idx)
                lst = self.tie_stages.setdefault(spec.key, [])
                if st not in lst:
                    lst.append(st)

    def _stage_of(self, idx: int) -> int:
        for s in range(self.num_stages):
            if self.parts[s] <= idx < self.parts[s + 1]:
                return s
        raise IndexError(idx)

    def _partition(self, method: str) -> List[int]:
        n, P = len(self.specs), self.num_stages
        if n < P:
            raise ValueError(f"{n} layers cannot fill {P} pipeline stages")
        m = method.lower()
        if m == "uniform":
            return partition_uniform(n, P)
        if m == "parameters":
            weights = [float(_count_params(s)) for s in self.specs]
            if sum(weights) == 0:
                return partition_uniform(n, P)
            return partition_balanced(weights, P)
        if m.startswith("type:"):
            pat = re.compile(method.split(":", 1)[1], re.IGNORECASE)

            def name(s: Any) -> str:
                return s.typename.__name__ if isinstance(s, LayerSpec) else type(s).__name__

            weights = [1.0 if pat.search(name(s)) else 0.0 for s in self.specs]
            if sum(weights) == 0:
                raise ValueError(f"partition_method {method!r} matches no layer")
            # zero-weight layers ride along; give them a tiny weight so parts stay contiguous
            return partition_balanced([w + 1e-6 for w in weights], P)
        raise NotImplementedError(f"partition_method {method!r}")

    def stage_layers(self) -> Tuple[int, int]:
        """[start, stop) indices of this stage's layers."""
        return self._local_start, self._local_stop

    def _run(self, start: int, stop: int, x: Any) -> Any:
        for f in self.forward_funcs[start:stop]:
            x = f(x)
        return x

    def forward(self, x: Any) -> Any:
        n = len(self.forward_funcs)
        k = self.activation_checkpoint_interval
        if k <= 0 or not self.training or not torch.is_grad_enabled():
            return self._run(0, n, x)
        from torch.utils.checkpoint import checkpoint

        for s in range(0, n, k):
            e = min(n, s + k)
            args = x if isinstance(x, tuple) else (x,)

            def chunk(*inp: Any, _s: int = s, _e: int = e) -> Any:
                return self._run(_s, _e, inp if len(inp) > 1 else inp[0])

            x = checkpoint(chunk, *args, use_reentrant=False)
        return x

    def layer_state_dicts(self) -> Dict[int, Dict[str, torch.Tensor]]:
        return {idx: m.state_dict() for idx, m in self._layer_modules.items()}

    def load_layer_state_dicts(self, states: Dict[int, Dict[str, torch.Tensor]],
                               strict: bool = True) -> None:
        loaded = set()
        for idx, m in sorted(self._layer_modules.items()):
            if id(m) in loaded:  # a tied module loads from its first (owning) layer index
                continue
            if idx in states:
                m.load_state_dict(states[idx], strict=strict)
                loaded.add(id(m))
            elif strict:
                raise KeyError(f"no state for pipeline layer {idx}")

    def tied_weights(self, key: str) -> List[torch.Tensor]:
        return [_get_attr(self.tied_modules[key], a) for a in self.tied_weight_attrs[key]]


# ---------------------------------------------------------------------------------- P2P
_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32,
           torch.bool, torch.uint8, torch.int8]
_META_LEN = 64


def _flatten(x: Activation) -> List[torch.Tensor]:
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (tuple, list)) and all(isinstance(t, torch.Tensor) for t in x):
        return list(x)
    raise TypeError("pipeline stage outputs must be a tensor or a tuple of tensors, got "
                    f"{type(x).__name__}")


class _Meta:
    def __init__(self, shapes: List[Tuple[int, ...]], dtypes: List[torch.dtype],
                 grads: List[bool], is_tuple: bool) -> None:
        self.shapes, self.dtypes, self.grads, self.is_tuple = shapes, dtypes, grads, is_tuple

    @classmethod
    def of(cls, x: Activation) -> "_Meta":
        ts = _flatten(x)
        return cls([tuple(t.shape) for t in ts], [t.dtype for t in ts],
                   [bool(t.requires_grad and t.is_floating_point()) for t in ts],
                   not isinstance(x, torch.Tensor))

    def encode(self, device: torch.device) -> torch.Tensor:
        v = [len(self.shapes), int(self.is_tuple)]
        for shp, dt, g in zip(self.shapes, self.dtypes, self.grads):
            v += [_DTYPES.index(dt), int(g), len(shp), *shp]
        if len(v) > _META_LEN:
            raise ValueError("pipeline activation metadata too large (too many tensors / dims)")
        return torch.tensor(v + [0] * (_META_LEN - len(v)), dtype=torch.int64, device=device)

    @classmethod
    def decode(cls, t: torch.Tensor) -> "_Meta":
        v = t.tolist()
        n, is_tuple, i = v[0], bool(v[1]), 2
        shapes, dtypes, grads = [], [], []
        for _ in range(n):
            dt, g, nd = v[i], v[i + 1], v[i + 2]
            shapes.append(tuple(v[i + 3:i + 3 + nd]))
            dtypes.append(_DTYPES[dt])
            grads.append(bool(g))
            i += 3 + nd
        return cls(shapes, dtypes, grads, is_tuple)

    def empty(self, device: torch.device) -> List[torch.Tensor]:
        return [torch.empty(s, dtype=d, device=device) for s, d in zip(self.shapes, self.dtypes)]


class _P2P:
    """Point-to-point transfers; gloo cannot send device tensors, so those stage through host."""

    def __init__(self, device: torch.device) -> None:
        self.device = device
        self.host_staging = dist.is_initialized() and dist.get_backend() == "gloo" and \
            device.type == "cuda"

    def run(self, sends: List[Tuple[torch.Tensor, int]], recvs: List[Tuple[torch.Tensor, int]]) -> None:
        if not sends and not recvs:
            return
        if self.host_staging:
            hs = [(t.cpu(), p) for t, p in sends]
            hr = [(torch.empty(t.shape, dtype=t.dtype), p) for t, p in recvs]
            self._exchange(hs, hr)
            for (t, _), (h, _) in zip(recvs, hr):
                t.copy_(h)
            return
        self._exchange([(t.contiguous(), p) for t, p in sends], recvs)

    @staticmethod
    def _exchange(sends: List[Tuple[torch.Tensor, int]], recvs: List[Tuple[torch.Tensor, int]]) -> None:
        ops = [dist.P2POp(dist.isend, t, p) for t, p in sends] + \
              [dist.P2POp(dist.irecv, t, p) for t, p in recvs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def __getattr__(name: str) -> Any:
    # the engine lives with the DeepSpeed-style engine it extends (avoids an import cycle)
    if name == "PipelineEngine":
        from determined_clone_amd.pytorch.deepspeed._pipe import PipelineEngine

        return PipelineEngine
    raise AttributeError(name)
