"""Fused flat-buffer optimizers (SGD, Adam/AdamW, LAMB) running the HIP kernels in
``ops/csrc/optim.hip``.

They subclass ``torch.optim.Optimizer`` and keep the user's ``param_groups`` (so LR schedulers,
``get_last_lr`` and ``state_dict`` round trips behave like torch's optimizers), but the state lives in
flat fp32 buffers parallel to the :class:`~determined_clone_amd.parallel.flat.FlatParamSpace`:

* low-precision (bf16/fp16) models get an fp32 MASTER copy; the kernel updates the master and writes
  the rounded model copy in the same pass;
* ``grad_scale`` / ``found_inf`` for AMP and the global clip coefficient are device tensors read by the
  kernel (no host synchronisation, unlike torch's GradScaler / ``clip_grad_norm_``);
* on CPU the same math runs through the PyTorch reference implementation (used by CPU tests).

Reference parity: the optimizers the reference trials construct (`torch.optim.SGD/Adam/AdamW`,
DeepSpeed FusedAdam/FusedLamb) and `PyTorchTrialContext.step_optimizer` clipping
(`harness/determined/pytorch/_pytorch_context.py:827`).
"""
import math
from typing import Any, Callable, Dict, List, Optional

import torch

from determined_clone_amd.ops import _ext, _grad
from determined_clone_amd.parallel.flat import FlatBuffer, FlatParamSpace


class _FlatState:
    """fp32 master + optimizer-state buffers for one dtype buffer."""

    def __init__(self, buf: FlatBuffer, names: List[str]) -> None:
        self.buf = buf
        if buf.dtype == torch.float32:
            self.master = buf.data
            self.model: Optional[torch.Tensor] = None
        else:
            self.master = buf.data.float()
            self.model = buf.data
        self.state = {n: torch.zeros(buf.numel, dtype=torch.float32, device=buf.device) for n in names}


def _as_groups(g: Any) -> List[Any]:
    """``norm_group``: None, one process group, or a list of them (pipeline x tensor parallel)."""
    if g is None:
        return []
    return list(g) if isinstance(g, (list, tuple)) else [g]


class FusedOptimizerBase(torch.optim.Optimizer):
    state_names: List[str] = []

    def __init__(self, params: Any, defaults: Dict[str, Any]) -> None:
        super().__init__(params, defaults)
        self.space = FlatParamSpace([g["params"] for g in self.param_groups],
                                    pad_multiple=self._pad_multiple())
        self.flat: Dict[torch.dtype, _FlatState] = self._build_flat_states()
        self._step = 0
        # Device-side [grad multiplier, found_inf, grad norm] produced by clip/unscale; None when
        # the step needs neither.
        self._dev_scale: Optional[torch.Tensor] = None
        # Host-side multiplier folded into every kernel (e.g. 1/world_size for summed all-reduce).
        self.grad_multiplier = 1.0
        self.last_grad_norm: Optional[torch.Tensor] = None
        # Device-resident per-group step hyper-parameters (lr, step-dependent terms) read by the
        # kernels instead of scalar launch arguments: a captured HIP graph then replays each step
        # with the current LR schedule (see pytorch/_graph.py). None = scalar arguments.
        self._dyn: Optional[torch.Tensor] = None
        # Pipeline parallelism (parallel/pipeline.py): the clip norm spans every stage, so the
        # squared norm is also summed over ``norm_group``; ``norm_exclude`` params (tied-weight
        # copies on non-owner stages) are left out so each tied weight is counted once.
        self.norm_group: Any = None
        self.norm_exclude: List[torch.Tensor] = []

    def _pad_multiple(self) -> int:
        return 1

    def _build_flat_states(self) -> Dict[torch.dtype, "_FlatState"]:
        return {dt: _FlatState(buf, self.state_names) for dt, buf in self.space.buffers.items()}

    # ------------------------------------------------------------------ grad preprocessing
    def prepare_grads(self, max_norm: float = 0.0, loss_scale: Optional[torch.Tensor] = None) -> None:
        """Compute (on device) the global grad norm, found_inf and the combined multiplier
        ``grad_multiplier / loss_scale * clip_coef`` consumed by the next :meth:`step`."""
        _grad.join()
        self.space.ensure_views()
        if self.norm_group is not None or self.norm_exclude:
            slices = [st.buf.grad[a:b] for st in self.flat.values()
                      for a, b in self._norm_ranges(st.buf, [(0, st.buf.grad.numel())])]
            groups = _as_groups(self.norm_group)
            self._finish_norm(self._sumsq(slices), max_norm, loss_scale, groups)
            return
        grads = [st.buf.grad for st in self.flat.values()]
        if grads and grads[0].is_cuda:
            self._dev_scale = _ext.load().grad_norm_scale(grads, loss_scale, self.grad_multiplier,
                                                          float(max_norm))
        else:
            sq = sum(float(g.float().pow(2).sum()) for g in grads)
            inv_ls = 1.0 / float(loss_scale[0]) if loss_scale is not None else 1.0
            mult = inv_ls * self.grad_multiplier
            norm = math.sqrt(sq) * mult if math.isfinite(sq) else float("inf")
            coef = 1.0
            if max_norm > 0 and math.isfinite(norm):
                coef = min(1.0, max_norm / (norm + 1e-6))
            inf = 0.0 if math.isfinite(sq) else 1.0
            dev = grads[0].device if grads else "cpu"
            self._dev_scale = torch.tensor([mult * coef, inf, norm], dtype=torch.float32, device=dev)
        self.last_grad_norm = self._dev_scale[2:3]

    def _norm_ranges(self, buf: FlatBuffer, ranges: List[Any]) -> List[Any]:
        """``ranges`` ([start, end) of ``buf``) minus the segments of ``norm_exclude`` params."""
        if not self.norm_exclude:
            return [(a, b) for a, b in ranges if b > a]
        ex = sorted((seg.offset, seg.offset + seg.numel) for p in self.norm_exclude
                    if self.space.buffer_of(p) is buf for seg in [self.space.segment(p)])
        out = []
        for a, b in ranges:
            cur = a
            for s, e in ex:
                if e <= cur or s >= b:
                    continue
                if s > cur:
                    out.append((cur, s))
                cur = max(cur, e)
            if cur < b:
                out.append((cur, b))
        return out

    def _sumsq(self, slices: List[torch.Tensor]) -> torch.Tensor:
        """Sum of squares of ``slices`` as a 1-element tensor (fp32 on GPU, fp64 on CPU)."""
        dev = next(iter(self.flat.values())).buf.grad.device if self.flat else torch.device("cpu")
        if dev.type == "cuda":
            if not slices:
                return torch.zeros(1, dtype=torch.float32, device=dev)
            return _ext.load().sumsq_partials(slices).sum().reshape(1)
        sq = torch.zeros(1, dtype=torch.float64)
        for s in slices:
            sq += s.double().pow(2).sum()
        return sq

    def _finish_norm(self, sq: torch.Tensor, max_norm: float, loss_scale: Optional[torch.Tensor],
                     groups: List[Any]) -> None:
        """All-reduce the squared norm over ``groups`` and derive ``_dev_scale``."""
        import torch.distributed as dist

        for g in groups:
            dist.all_reduce(sq, group=g)
        if sq.is_cuda:
            self._dev_scale = _ext.load().norm_finalize(sq, loss_scale, self.grad_multiplier,
                                                        float(max_norm))
        else:
            tot = float(sq)
            inv_ls = 1.0 / float(loss_scale[0]) if loss_scale is not None else 1.0
            mult = inv_ls * self.grad_multiplier
            finite = math.isfinite(tot)
            norm = math.sqrt(tot) * mult if finite else float("inf")
            coef = min(1.0, max_norm / (norm + 1e-6)) if max_norm > 0 and finite else 1.0
            self._dev_scale = torch.tensor([mult * coef, 0.0 if finite else 1.0, norm],
                                           dtype=torch.float32)
        self.last_grad_norm = self._dev_scale[2:3]

    @property
    def found_inf(self) -> Optional[torch.Tensor]:
        return None if self._dev_scale is None else self._dev_scale[1:2]

    def zero_grad(self, set_to_none: bool = False) -> None:  # type: ignore[override]
        # Flat gradients are zeroed in one memset per dtype; views stay installed.
        self.space.zero_grad()

    # ------------------------------------------------------------------ HIP-graph support
    graph_capturable = True

    def _dyn_row(self, group: Dict[str, Any], step: int) -> List[float]:
        """Per-group values the kernels read from the device buffer for optimizer step ``step``."""
        return [float(group["lr"]), 0.0, 0.0, 0.0]

    def enable_device_hparams(self) -> None:
        dev = next(iter(self.flat.values())).master.device if self.flat else torch.device("cpu")
        if dev.type != "cuda":
            return
        self._dyn = torch.zeros(len(self.param_groups), 4, dtype=torch.float32, device=dev)

    def refresh_device_hparams(self, step: Optional[int] = None) -> None:
        """Upload this step's lr / bias-correction terms (an async H2D copy from pinned memory,
        issued OUTSIDE any captured graph)."""
        if self._dyn is None:
            return
        step = self._step if step is None else step
        rows = [self._dyn_row(g, step) for g in self.param_groups]
        self._dyn.copy_(torch.tensor(rows, dtype=torch.float32).pin_memory(), non_blocking=True)

    def _dyn_of(self, group: Dict[str, Any]) -> Optional[torch.Tensor]:
        if self._dyn is None:
            return None
        for i, g in enumerate(self.param_groups):
            if g is group:
                return self._dyn[i]
        return None

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure: Optional[Callable] = None) -> Any:  # type: ignore[override]
        loss = closure() if closure is not None else None
        _grad.join()
        self.space.ensure_views()
        self._step += 1
        if self._dyn is not None and not torch.cuda.is_current_stream_capturing():
            self.refresh_device_hparams()
        dev_scale = self._dev_scale
        for st in self.flat.values():
            for gi, (start, end) in st.buf.group_ranges.items():
                if end <= start:
                    continue
                self._step_range(st, self.param_groups[gi], start, end, dev_scale)
        self._dev_scale = None
        return loss

    def _slice(self, t: Optional[torch.Tensor], start: int, end: int) -> Optional[torch.Tensor]:
        return None if t is None else t[start:end]

    def _step_range(self, st: _FlatState, group: Dict[str, Any], start: int, end: int,
                    dev_scale: Optional[torch.Tensor]) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------ state dict
    def state_dict(self) -> Dict[str, Any]:  # type: ignore[override]
        """torch-compatible layout: per-param state keyed by flattened param index, plus the fp32
        master copy for low-precision models (`master_param`)."""
        packed_groups = []
        index = 0
        for g in self.param_groups:
            pg = {k: v for k, v in g.items() if k != "params"}
            pg["params"] = list(range(index, index + len(g["params"])))
            index += len(g["params"])
            packed_groups.append(pg)
        state: Dict[int, Dict[str, Any]] = {}
        for st in self.flat.values():
            for seg in st.buf.segments:
                s: Dict[str, Any] = {"step": torch.tensor(float(self._step))}
                for n in self.state_names:
                    s[n] = st.buf.view(st.state[n], seg).clone()
                if st.model is not None:
                    s["master_param"] = st.buf.view(st.master, seg).clone()
                state[seg.index] = s
        return {"state": state, "param_groups": packed_groups}

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:  # type: ignore[override]
        groups = state_dict["param_groups"]
        if len(groups) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        for g, saved in zip(self.param_groups, groups):
            for k, v in saved.items():
                if k != "params":
                    g[k] = v
        state = {int(k): v for k, v in state_dict["state"].items()}
        if state and not any("step" in s for s in state.values()):
            self._step = max(self._step, 1)  # torch SGD keeps no step count
        with torch.no_grad():
            for st in self.flat.values():
                for seg in st.buf.segments:
                    s = state.get(seg.index)
                    if not s:
                        continue
                    for n in self.state_names:
                        src = s.get(n, s.get(self._torch_alias(n)))
                        if src is not None:
                            st.buf.view(st.state[n], seg).copy_(src)
                    if "step" in s:
                        self._step = int(float(s["step"]))
                    if st.model is not None:
                        mp = s.get("master_param")
                        if mp is not None:
                            st.buf.view(st.master, seg).copy_(mp)
                        else:
                            st.buf.view(st.master, seg).copy_(seg.param.data.float())

    def _torch_alias(self, name: str) -> str:
        return name

    def sync_master_from_model(self) -> None:
        """After the model weights were loaded/overwritten (e.g. checkpoint restore or broadcast
        from rank 0), refresh the fp32 master copies."""
        with torch.no_grad():
            for st in self.flat.values():
                if st.model is not None:
                    st.master.copy_(st.model.float())


class FusedSGD(FusedOptimizerBase):
    state_names = ["momentum_buffer"]

    def _dyn_row(self, group: Dict[str, Any], step: int) -> List[float]:
        return [float(group["lr"]), 1.0 if step == 1 else 0.0, 0.0, 0.0]

    def __init__(self, params: Any, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False) -> None:
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults)

    def _step_range(self, st, group, start, end, dev_scale) -> None:
        self._update(st.master[start:end], self._slice(st.model, start, end),
                     st.buf.grad[start:end], {n: v[start:end] for n, v in st.state.items()},
                     group, dev_scale)

    def _update(self, master, model, grad, states, group, dev_scale) -> None:
        """One fused SGD pass over matching slices (flat range or ZeRO shard piece)."""
        mom = states["momentum_buffer"]
        first = self._step == 1
        if master.is_cuda:
            _ext.load().sgd(master, model, grad, mom, group["lr"], group["momentum"],
                            group["dampening"], group["weight_decay"], group["nesterov"], first,
                            self.grad_multiplier if dev_scale is None else 1.0, dev_scale,
                            self._dyn_of(group))
            return
        if dev_scale is not None and float(dev_scale[1]) != 0.0:
            return
        gs = float(dev_scale[0]) if dev_scale is not None else self.grad_multiplier
        g = grad.float() * gs
        wd, m = group["weight_decay"], group["momentum"]
        if wd:
            g = g + wd * master
        if m:
            if first:
                mom.copy_(g)
            else:
                mom.mul_(m).add_(g, alpha=1 - group["dampening"])
            g = g + m * mom if group["nesterov"] else mom
        master.add_(g, alpha=-group["lr"])
        if model is not None:
            model.copy_(master)


class FusedAdam(FusedOptimizerBase):
    state_names = ["exp_avg", "exp_avg_sq"]

    def _dyn_row(self, group: Dict[str, Any], step: int) -> List[float]:
        b1, b2 = group["betas"]
        return [float(group["lr"]), 1.0 - b1 ** step, 1.0 - b2 ** step, 0.0]

    def __init__(self, params: Any, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = False) -> None:
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        self.adamw = adamw
        super().__init__(params, defaults)

    def _step_range(self, st, group, start, end, dev_scale) -> None:
        self._update(st.master[start:end], self._slice(st.model, start, end),
                     st.buf.grad[start:end], {n: v[start:end] for n, v in st.state.items()},
                     group, dev_scale)

    def _update(self, master, model, grad, states, group, dev_scale) -> None:
        """One fused Adam/AdamW pass over matching slices (flat range or ZeRO shard piece)."""
        m, v = states["exp_avg"], states["exp_avg_sq"]
        b1, b2 = group["betas"]
        if master.is_cuda:
            _ext.load().adam(master, model, grad, m, v, group["lr"], b1, b2, group["eps"],
                             group["weight_decay"], self.adamw, self._step,
                             self.grad_multiplier if dev_scale is None else 1.0, dev_scale,
                             self._dyn_of(group))
            return
        if dev_scale is not None and float(dev_scale[1]) != 0.0:
            return
        gs = float(dev_scale[0]) if dev_scale is not None else self.grad_multiplier
        g = grad.float() * gs
        lr, wd = group["lr"], group["weight_decay"]
        if self.adamw:
            master.mul_(1 - lr * wd)
        elif wd:
            g = g + wd * master
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** self._step
        bc2 = 1 - b2 ** self._step
        denom = (v.sqrt() / math.sqrt(bc2)).add_(group["eps"])
        master.addcdiv_(m, denom, value=-lr / bc1)
        if model is not None:
            model.copy_(master)


class FusedAdamW(FusedAdam):
    def __init__(self, params: Any, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2) -> None:
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=True)


class FusedLAMB(FusedOptimizerBase):
    """LAMB (You et al. 2019): Adam update + decoupled decay, scaled per tensor by
    ||w|| / ||update||. Per-tensor norms come from a chunk table over the flat buffer."""

    graph_capturable = False  # scalar-argument path only
    state_names = ["exp_avg", "exp_avg_sq"]
    CHUNK = 65536

    def __init__(self, params: Any, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-6,
                 weight_decay: float = 0.01) -> None:
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables: Dict[Any, Any] = {}

    def _table(self, st: _FlatState, start: int, end: int):
        key = (st.buf.dtype, start, end)
        if key in self._tables:
            return self._tables[key]
        cstart, clen, cseg, seg_begin = [], [], [], [0]
        segs = [s for s in st.buf.segments if start <= s.offset < end]
        for si, seg in enumerate(segs):
            off = seg.offset - start
            for c in range(0, seg.numel, self.CHUNK):
                cstart.append(off + c)
                clen.append(min(self.CHUNK, seg.numel - c))
                cseg.append(si)
            seg_begin.append(len(cstart))
        dev = st.master.device
        t = (torch.tensor(cstart, dtype=torch.int64, device=dev),
             torch.tensor(clen, dtype=torch.int32, device=dev),
             torch.tensor(cseg, dtype=torch.int32, device=dev),
             torch.tensor(seg_begin, dtype=torch.int32, device=dev), segs)
        self._tables[key] = t
        return t

    def _step_range(self, st, group, start, end, dev_scale) -> None:
        master = st.master[start:end]
        grad = st.buf.grad[start:end]
        m = st.state["exp_avg"][start:end]
        v = st.state["exp_avg_sq"][start:end]
        model = self._slice(st.model, start, end)
        b1, b2 = group["betas"]
        cstart, clen, cseg, seg_begin, segs = self._table(st, start, end)
        if master.is_cuda:
            ubuf = torch.empty_like(master)
            _ext.load().lamb(master, model, grad, m, v, ubuf, cstart, clen, cseg, seg_begin,
                             group["lr"], b1, b2, group["eps"], group["weight_decay"], self._step,
                             self.grad_multiplier if dev_scale is None else 1.0, dev_scale)
            return
        if dev_scale is not None and float(dev_scale[1]) != 0.0:
            return
        gs = float(dev_scale[0]) if dev_scale is not None else self.grad_multiplier
        bc1 = 1 - b1 ** self._step
        bc2 = 1 - b2 ** self._step
        for seg in segs:
            sl = slice(seg.offset - start, seg.offset - start + seg.numel)
            w, g = master[sl], grad[sl].float() * gs
            m[sl].mul_(b1).add_(g, alpha=1 - b1)
            v[sl].mul_(b2).addcmul_(g, g, value=1 - b2)
            u = (m[sl] / bc1) / ((v[sl] / bc2).sqrt() + group["eps"]) + group["weight_decay"] * w
            wn, un = w.norm(), u.norm()
            ratio = (wn / un) if (wn > 0 and un > 0) else torch.tensor(1.0)
            w.add_(u * (-group["lr"] * float(ratio)))
        if model is not None:
            model.copy_(master)


class DeviceGradScaler:
    """Dynamic loss scaling kept entirely on the device (no ``.item()`` per step).

    API mirrors ``torch.cuda.amp.GradScaler``: ``scale(loss)``, ``step(opt)``, ``update()``,
    ``state_dict``/``load_state_dict`` (reference: `PyTorchTrialContext.wrap_scaler`)."""

    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000,
                 device: Optional[torch.device] = None, enabled: bool = True) -> None:
        dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.state = torch.tensor([init_scale, 0.0], dtype=torch.float32, device=dev)
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        self._enabled = enabled
        self._last_dev_scale: Optional[torch.Tensor] = None

    def is_enabled(self) -> bool:
        return self._enabled

    def get_scale(self) -> float:
        return float(self.state[0])

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        if not self._enabled:
            return loss
        return loss * self.state[0].to(loss.dtype)

    def unscale_(self, optimizer: FusedOptimizerBase, max_norm: float = 0.0) -> None:
        optimizer.prepare_grads(max_norm=max_norm, loss_scale=self.state[0:1] if self._enabled else None)
        self._last_dev_scale = optimizer._dev_scale

    def step(self, optimizer: FusedOptimizerBase, max_norm: float = 0.0) -> None:
        if optimizer._dev_scale is None:
            self.unscale_(optimizer, max_norm)
        self._last_dev_scale = optimizer._dev_scale
        optimizer.step()

    def update(self) -> None:
        if not self._enabled or self._last_dev_scale is None:
            return
        ds = self._last_dev_scale
        if self.state.is_cuda:
            _ext.load().amp_scaler_update(self.state, ds, self.growth_factor, self.backoff_factor,
                                          self.growth_interval)
        else:
            if float(ds[1]) != 0.0:
                self.state[0] *= self.backoff_factor
                self.state[1] = 0.0
            else:
                self.state[1] += 1
                if self.state[1] >= self.growth_interval:
                    self.state[0] *= self.growth_factor
                    self.state[1] = 0.0
        self._last_dev_scale = None

    def state_dict(self) -> Dict[str, Any]:
        return {"scale": float(self.state[0]), "growth_tracker": int(self.state[1]),
                "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.state[0] = sd["scale"]
        self.state[1] = sd.get("growth_tracker", 0)
        self.growth_factor = sd.get("growth_factor", self.growth_factor)
        self.backoff_factor = sd.get("backoff_factor", self.backoff_factor)
        self.growth_interval = sd.get("growth_interval", self.growth_interval)


def fuse_optimizer(opt: torch.optim.Optimizer) -> Optional[FusedOptimizerBase]:
    """Build the fused equivalent of a torch optimizer (same param groups / hyperparameters), or
    None if there is no fused equivalent (the caller then keeps the user's optimizer)."""
    if isinstance(opt, FusedOptimizerBase):
        return opt
    groups = []
    for g in opt.param_groups:
        groups.append(dict(g))
    if type(opt) is torch.optim.SGD:
        if any(g.get("maximize") for g in groups):
            return None
        new: FusedOptimizerBase = FusedSGD(groups, lr=groups[0]["lr"])
    elif type(opt) in (torch.optim.Adam, torch.optim.AdamW):
        if any(g.get("amsgrad") or g.get("maximize") for g in groups):
            return None
        cls = FusedAdamW if type(opt) is torch.optim.AdamW else FusedAdam
        new = cls(groups, lr=groups[0]["lr"])
    else:
        return None
    if opt.state:
        new.load_state_dict(_convert_torch_state(opt))
    return new


def _convert_torch_state(opt: torch.optim.Optimizer) -> Dict[str, Any]:
    sd = opt.state_dict()
    return sd
