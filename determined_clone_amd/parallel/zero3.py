"""ZeRO stage 3: parameters partitioned over the data-parallel group, gathered per module on use.

The reference reaches ZeRO-3 through DeepSpeed (``zero_optimization.stage: 3`` in
`examples/hf_trainer_api/*/ds_configs/ds_config_stage_3.json`, DeepSpeedTrial engines built by
`harness/determined/pytorch/deepspeed/_deepspeed_context.py:178`). Design here (MI355X-first: few,
large RCCL collectives on flat buffers):

* **Units.** The model is cut into units: every element of the outermost ``nn.ModuleList`` /
  ``nn.Sequential`` containers (transformer blocks, ResNet stages' blocks) plus a root unit with
  the remaining parameters (embeddings, final norm, head). Each unit's parameters of one
  (optimizer group, dtype) live in ONE flat buffer whose rank-``r`` slice (1/W, 64-element
  aligned) is the only persistent copy: an ``nn.Parameter`` the fused optimizer owns (fp32 master
  + Adam/SGD state for the shard only).
* **Forward.** A pre-forward hook all-gathers the unit's flat buffer
  (``all_gather_into_tensor``, one collective per unit) into storage that is re-allocated on
  demand; the module's parameters are views into it. A post-forward hook frees the storage
  (``untyped_storage().resize_(0)``; autograd's saved views keep their metadata and see the data
  again once it is re-gathered). The root unit stays resident from forward until its gradients
  are reduced.
* **Backward.** A hook on the unit's outputs re-gathers the parameters just before the unit's
  backward and installs ``.grad`` views into a zeroed flat gradient buffer (marked for the fused
  kernels' in-place gradient accumulation, ``ops/_grad.py``). When every parameter of the unit
  has accumulated (post-accumulate hooks), one ``reduce_scatter_tensor`` sums the flat gradient
  into the shard's gradient -- asynchronously, at most two units in flight -- and the full
  parameters and gradients are freed.
* **Step.** The fused optimizer updates the shards (clip norm all-reduced over the group);
  the next forward gathers the updated shards.

Peak memory per rank: shards of everything + the live units' full parameters/gradients, i.e. the
model no longer has to fit one GPU. ``full_state_dict()`` gathers a consolidated copy for
checkpoints (``stage3_gather_16bit_weights_on_model_save``).
"""
import logging
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from determined_clone_amd.ops import _grad
from determined_clone_amd.parallel import _caps
from determined_clone_amd.parallel.flat import ALIGN

logger = logging.getLogger("determined_clone_amd.parallel.zero3")


class _Unit:
    def __init__(self, name: str, module: nn.Module, params: List[nn.Parameter], group_idx: int,
                 pg: Any, world: int, rank: int, root: bool) -> None:
        self.name = name
        self.module = module
        self.params = params
        self.group_idx = group_idx
        self.pg, self.world, self.rank, self.root = pg, world, rank, root
        self.dtype = params[0].dtype
        self.device = params[0].device
        self.numels = [p.numel() for p in params]
        total = sum(self.numels)
        q = world * ALIGN
        self.padded = (total + q - 1) // q * q
        self.shard_numel = self.padded // world
        self.esz = torch.empty(0, dtype=self.dtype).element_size()
        self.full = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
        off = 0
        self.offsets = []
        with torch.no_grad():
            for p, n in zip(params, self.numels):
                self.full[off:off + n].copy_(p.data.reshape(-1))
                self.offsets.append(off)
                off += n
        s0 = rank * self.shard_numel
        self.shard = nn.Parameter(self.full[s0:s0 + self.shard_numel].clone())
        for p, o, n in zip(params, self.offsets, self.numels):
            p.data = self.full[o:o + n].view(p.shape)
        self.full_grad: Optional[torch.Tensor] = None
        self.gathered = True
        self.pending = len(params)
        self.in_backward = False
        self.release()

    # ------------------------------------------------------------------ parameters
    def gather(self) -> None:
        if self.gathered:
            return
        self.full.untyped_storage().resize_(self.padded * self.esz)
        if self.world > 1:
            if _caps.tensor_collectives(self.pg, self.full.device):
                dist.all_gather_into_tensor(self.full, self.shard.data, group=self.pg)
            else:  # gloo on device tensors: list form
                n = self.shard_numel
                outs = [self.full[r * n:(r + 1) * n] for r in range(self.world)]
                dist.all_gather(outs, self.shard.data.clone(), group=self.pg)
        else:
            self.full.copy_(self.shard.data)
        self.gathered = True

    def release(self) -> None:
        if self.gathered:
            self.full.untyped_storage().resize_(0)
            self.gathered = False

    # ------------------------------------------------------------------ gradients
    def begin_backward(self) -> None:
        self.gather()
        if self.in_backward:
            return
        self.in_backward = True
        self.pending = len(self.params)
        if self.full_grad is None:
            self.full_grad = torch.zeros(self.padded, dtype=self.dtype, device=self.device)
        for p, o, n in zip(self.params, self.offsets, self.numels):
            p.grad = self.full_grad[o:o + n].view(p.shape)
            p._dca_direct_grad = True

    def detach_grads(self) -> torch.Tensor:
        g = self.full_grad
        for p in self.params:
            p.grad = None
            p._dca_direct_grad = False
        self.full_grad = None
        self.in_backward = False
        return g


class Zero3Partitioner:
    """Partitions ``model``'s parameters over ``group``; ``param_groups`` (lists of model params,
    one per optimizer group) decide which shards share optimizer hyper-parameters."""

    MAX_IN_FLIGHT = 2

    def __init__(self, model: nn.Module, param_groups: List[List[nn.Parameter]],
                 group: Any = None) -> None:
        self.model = model
        self.pg = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        gid = {}
        for i, ps in enumerate(param_groups):
            for p in ps:
                gid[id(p)] = i
        self.units: List[_Unit] = []
        self._by_module: Dict[int, List[_Unit]] = {}
        claimed = set()
        for name, mod in self._unit_modules(model):
            self._add_units(name, mod, list(mod.parameters()), gid, claimed, root=False)
        root_params = [p for p in model.parameters() if id(p) not in claimed]
        self._add_units("<root>", model, root_params, gid, claimed, root=True)
        self._inflight: List[Tuple[Any, torch.Tensor, torch.Tensor, _Unit]] = []
        self._handles = []
        for mod_id, units in self._by_module.items():
            mod = units[0].module
            self._handles.append(mod.register_forward_pre_hook(self._pre_forward(units)))
            self._handles.append(mod.register_forward_hook(self._post_forward(units)))
        for u in self.units:
            for p in u.params:
                self._handles.append(p.register_post_accumulate_grad_hook(self._on_grad(u)))
        n_full = sum(u.padded for u in self.units)
        logger.info(f"ZeRO-3: {len(self.units)} units, {n_full / 1e6:.1f}M parameters, "
                    f"{n_full // self.world / 1e6:.1f}M per rank (world {self.world})")

    @staticmethod
    def _unit_modules(model: nn.Module) -> List[Tuple[str, nn.Module]]:
        out: List[Tuple[str, nn.Module]] = []

        def visit(prefix: str, m: nn.Module) -> None:
            for name, child in m.named_children():
                full = f"{prefix}{name}"
                if isinstance(child, (nn.ModuleList, nn.Sequential)):
                    for n2, c2 in child.named_children():
                        if any(True for _ in c2.parameters()):
                            out.append((f"{full}.{n2}", c2))
                else:
                    visit(full + ".", child)

        visit("", model)
        return out

    def _add_units(self, name: str, mod: nn.Module, params: List[nn.Parameter], gid: Dict[int, int],
                   claimed: set, root: bool) -> None:
        buckets: Dict[Tuple[int, torch.dtype], List[nn.Parameter]] = {}
        for p in params:
            if id(p) in claimed or not p.requires_grad:
                continue
            claimed.add(id(p))
            if id(p) not in gid:
                continue  # not optimised: stays a plain, unpartitioned parameter
            buckets.setdefault((gid[id(p)], p.dtype), []).append(p)
        for (g, _), ps in sorted(buckets.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            u = _Unit(name, mod, ps, g, self.pg, self.world, self.rank, root)
            self.units.append(u)
            self._by_module.setdefault(id(mod), []).append(u)

    # ------------------------------------------------------------------ optimizer view
    def shard_param_groups(self, num_groups: int) -> List[List[nn.Parameter]]:
        out: List[List[nn.Parameter]] = [[] for _ in range(num_groups)]
        for u in self.units:
            out[u.group_idx].append(u.shard)
        return out

    # ------------------------------------------------------------------ hooks
    def _pre_forward(self, units: List[_Unit]):
        def hook(mod: nn.Module, args: Any) -> None:
            for u in units:
                u.gather()
        return hook

    def _post_forward(self, units: List[_Unit]):
        def hook(mod: nn.Module, args: Any, output: Any) -> Any:
            grad_on = torch.is_grad_enabled()
            if grad_on:
                tensors = [t for t in _tensors(output) if t.requires_grad]
                for t in tensors:
                    t.register_hook(self._pre_backward(units))
            for u in units:
                if not u.root or not grad_on:
                    u.release()
            return None
        return hook

    def _pre_backward(self, units: List[_Unit]):
        def hook(grad: torch.Tensor) -> None:
            for u in units:
                u.begin_backward()
            return None
        return hook

    def _on_grad(self, u: _Unit):
        def hook(p: torch.Tensor) -> None:
            if p.is_cuda:
                _grad.join()  # side-stream weight gradients (ops/_grad.py) land before reducing
            if not u.in_backward:
                # gradient produced without the output hook (e.g. a parameter used outside its
                # unit's forward): adopt it into the unit's gradient buffer
                g = p.grad
                u.begin_backward()
                if g is not None and p.grad is not g:
                    p.grad.add_(g)
            u.pending -= 1
            if u.pending == 0:
                self._reduce(u)
        return hook

    def _reduce(self, u: _Unit) -> None:
        while len(self._inflight) >= self.MAX_IN_FLIGHT:
            self._complete(self._inflight.pop(0))
        full_grad = u.detach_grads()
        u.release()
        if self.world > 1:
            n = u.shard_numel
            if _caps.tensor_collectives(self.pg, full_grad.device):
                out = torch.empty(n, dtype=full_grad.dtype, device=full_grad.device)
                work = dist.reduce_scatter_tensor(out, full_grad, op=dist.ReduceOp.SUM,
                                                  group=self.pg, async_op=True)
            else:  # gloo on device tensors: all-reduce and keep the own slice
                work = dist.all_reduce(full_grad, op=dist.ReduceOp.SUM, group=self.pg,
                                       async_op=True)
                out = full_grad[u.rank * n:(u.rank + 1) * n]
            self._inflight.append((work, out, full_grad, u))
        else:
            self._complete((None, full_grad, full_grad, u))

    @staticmethod
    def _complete(item: Tuple[Any, torch.Tensor, torch.Tensor, _Unit]) -> None:
        work, out, _full, u = item
        if work is not None:
            work.wait()
        if u.shard.grad is None:
            u.shard.grad = out.clone()
        else:
            u.shard.grad.add_(out)

    def finish_backward(self) -> None:
        """After ``loss.backward()``: reduce units whose gradients never completed (unused
        parameters), drain the in-flight reduce-scatters, free the root unit."""
        for u in self.units:
            if u.in_backward:
                self._reduce(u)
        while self._inflight:
            self._complete(self._inflight.pop(0))
        for u in self.units:
            u.release()

    # ------------------------------------------------------------------ consolidated state
    @torch.no_grad()
    def full_state_dict(self) -> Dict[str, torch.Tensor]:
        """Consolidated module state (every rank participates; every rank gets the copy)."""
        for u in self.units:
            u.gather()
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        for u in self.units:
            u.release()
        return sd

    @torch.no_grad()
    def load_full_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        for u in self.units:
            u.gather()
        self.model.load_state_dict(sd, strict=strict)
        for u in self.units:
            s0 = u.rank * u.shard_numel
            u.shard.data.copy_(u.full[s0:s0 + u.shard_numel])
            u.release()

    def optimizer_param_units(self, num_groups: int) -> List[_Unit]:
        """Units in the optimizer's flattened parameter order (group by group, as
        :meth:`shard_param_groups` lays them out): state index i belongs to unit i of this list."""
        out: List[_Unit] = []
        for g in range(num_groups):
            out.extend(u for u in self.units if u.group_idx == g)
        return out

    def reshard_optimizer_state(self, saved: List[Dict[str, Any]], num_groups: int) -> Dict[str, Any]:
        """Build THIS rank's optimizer state dict from the per-rank shard state dicts written at
        another data-parallel size. A unit's flat layout depends on the world size only through
        the tail padding, so the old shards are concatenated, cut to the unit's true numel,
        re-padded for the current world size and sliced at this rank's offset."""
        units = self.optimizer_param_units(num_groups)
        old = [{int(k): v for k, v in sd["state"].items()} for sd in saved]
        state: Dict[int, Dict[str, Any]] = {}
        for i, u in enumerate(units):
            parts = [o.get(i) for o in old]
            if any(p is None for p in parts):
                continue
            total = sum(u.numels)
            s0 = u.rank * u.shard_numel
            new: Dict[str, Any] = {}
            for key, v0 in parts[0].items():
                if torch.is_tensor(v0) and v0.dim() == 1:
                    flat = torch.cat([p[key].reshape(-1) for p in parts])[:total]
                    full = torch.zeros(u.padded, dtype=v0.dtype)
                    full[:total].copy_(flat)
                    new[key] = full[s0:s0 + u.shard_numel].clone()
                else:
                    new[key] = v0
            state[i] = new
        return {"state": state, "param_groups": saved[0]["param_groups"]}

    def remove_hooks(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []


def _tensors(x: Any) -> List[torch.Tensor]:
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (tuple, list)):
        return [t for e in x for t in _tensors(e)]
    if isinstance(x, dict):
        return [t for e in x.values() for t in _tensors(e)]
    return []
