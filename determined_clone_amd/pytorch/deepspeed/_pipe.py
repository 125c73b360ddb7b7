"""Pipeline-parallel DeepSpeed-style engine: 1F1B schedule over stage-to-stage P2P.

See :mod:`determined_clone_amd.parallel.pipeline` for the design (layer specs, partitioning,
grid, schedule); reference: `harness/determined/pytorch/deepspeed/_deepspeed_context.py:188`.
"""
import logging
import pathlib
from typing import Any, Dict, Iterator, List, Optional, Tuple, Union

import torch
import torch.distributed as dist

from determined_clone_amd.ops import _grad
from determined_clone_amd.parallel.pipeline import (_META_LEN, Activation, PipelineModule, _flatten,
                                                    _Meta, _P2P)
from determined_clone_amd.pytorch.deepspeed._engine import DeepSpeedEngine

logger = logging.getLogger("determined_clone_amd.parallel.pipeline")


# ---------------------------------------------------------------------------------- engine
class PipelineEngine(DeepSpeedEngine):
    """DeepSpeed ``PipelineEngine`` surface: ``train_batch(data_iter)`` / ``eval_batch(data_iter)``
    each consume ``gradient_accumulation_steps`` micro-batches ``(inputs, labels)`` from the
    iterator (first stage uses inputs, last stage labels; middle stages pass ``None``). The
    batch-size arithmetic (``train_batch_size = micro * accumulation * data_parallel_size``) uses
    the data-parallel size, not the world size."""

    def __init__(self, model: PipelineModule, config: Any, optimizer: Any = None,
                 model_parameters: Any = None, lr_scheduler: Any = None,
                 device: Optional[torch.device] = None) -> None:
        if not isinstance(model, PipelineModule):
            raise TypeError("PipelineEngine requires a PipelineModule")
        self.grid = model._grid
        grid = self.grid
        super().__init__(model, config, optimizer=optimizer, model_parameters=model_parameters,
                         lr_scheduler=lr_scheduler, group=grid.dp_group, device=device)
        if self.config.fp16 and self.scaler is not None:
            raise ValueError("pipeline parallelism does not support fp16 dynamic loss scaling; "
                             "use bf16 (or a static fp16 loss_scale)")
        self.num_stages = grid.pipe_parallel_size
        self.stage_id = grid.stage_id
        self.micro_batches = self.config.grad_accum
        self.is_first = self.stage_id == 0
        self.is_last = self.stage_id == self.num_stages - 1
        self.prev_rank = grid.stage_to_global(self.stage_id - 1) if not self.is_first else None
        self.next_rank = grid.stage_to_global(self.stage_id + 1) if not self.is_last else None
        self._p2p = _P2P(self.device)
        self._tie_groups: Dict[str, Tuple[Any, List[int]]] = {}
        self._setup_ties()
        norm_groups = [grid.pp_group] if self.num_stages > 1 else []
        if grid.model_parallel_size > 1:
            # tensor parallelism inside each stage (parallel/tensor.py): sharded parameters are
            # summed over the TP group too, replicated ones counted on TP rank 0 only
            from determined_clone_amd.parallel import tensor as tp

            norm_groups.append(grid.mp_group)
            if grid.model_parallel_id != 0:
                self.optimizer.norm_exclude = list(self.optimizer.norm_exclude) + \
                    tp.replicated_params(list(model.parameters()))
            self.mp_rank = grid.model_parallel_id
        if norm_groups:
            self.optimizer.norm_group = norm_groups if len(norm_groups) > 1 else norm_groups[0]
        self.agg_train_loss: Optional[torch.Tensor] = None
        self.first_output_send = True

    # ------------------------------------------------------------------ tied weights
    def _setup_ties(self) -> None:
        mod: PipelineModule = self.module
        if not dist.is_initialized() or self.grid.world_size == 1:
            return
        exclude: List[torch.Tensor] = []
        for key in sorted(mod.tie_stages):
            stages = sorted(mod.tie_stages[key])
            if len(stages) < 2:
                continue
            for d in range(self.grid.data_parallel_size):  # collective: same order on every rank
                for m in range(self.grid.model_parallel_size):  # one tie group per TP rank
                    ranks = [self.grid.stage_to_global(s, d, m) for s in stages]
                    g = dist.new_group(ranks)
                    if self.grid.global_rank in ranks:
                        self._tie_groups[key] = (g, ranks)
            if key in self._tie_groups:
                g, ranks = self._tie_groups[key]
                for w in mod.tied_weights(key):
                    self._bcast(w.data, ranks[0], g)
                if self.stage_id != stages[0]:
                    exclude += mod.tied_weights(key)
        self.optimizer.norm_exclude = exclude
        if exclude or self._tie_groups:
            self.optimizer.sync_master_from_model()

    def _bcast(self, t: torch.Tensor, src: int, group: Any) -> None:
        if self._p2p.host_staging:
            h = t.cpu()
            dist.broadcast(h, src, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, src, group=group)

    def _allreduce(self, t: torch.Tensor, group: Any) -> None:
        if self._p2p.host_staging:
            h = t.cpu()
            dist.all_reduce(h, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=group)

    def _reduce_tied_grads(self) -> None:
        if self.device.type == "cuda":
            _grad.join()  # tied weights' side-stream gradients (ops/_grad.py) land before the reduce
        self.optimizer.space.ensure_views()
        for key, (g, _) in self._tie_groups.items():
            for w in self.module.tied_weights(key):
                if w.grad is not None:
                    self._allreduce(w.grad, g)

    # ------------------------------------------------------------------ data
    def _next_batch(self, data_iter: Optional[Iterator[Any]]) -> Tuple[Any, Any]:
        if data_iter is None:
            raise ValueError(f"pipeline stage {self.stage_id} needs the data iterator "
                             "(first stage: inputs, last stage: labels)")
        batch = next(data_iter)
        if isinstance(batch, dict):
            inputs, labels = batch.get("inputs"), batch.get("labels")
        elif isinstance(batch, (tuple, list)) and len(batch) == 2:
            inputs, labels = batch
        else:
            raise ValueError("pipeline micro-batches must be (inputs, labels) pairs")
        return self._to_device(inputs), self._to_device(labels)

    def _to_device(self, x: Any) -> Any:
        if isinstance(x, torch.Tensor):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (tuple, list)):
            return type(x)(self._to_device(t) for t in x)
        return x

    # ------------------------------------------------------------------ P2P helpers
    def _send_meta(self, y: Activation) -> None:
        meta = _Meta.of(y)
        self._p2p.run([(meta.encode(self.device), self.next_rank)], [])
        self._out_meta = meta

    def _recv_meta(self) -> None:
        buf = torch.zeros(_META_LEN, dtype=torch.int64, device=self.device)
        self._p2p.run([], [(buf, self.prev_rank)])
        self._in_meta = _Meta.decode(buf.cpu())

    def _act_tensors(self, y: Activation) -> List[torch.Tensor]:
        return [t.detach() for t in _flatten(y)]

    def _new_input(self) -> List[torch.Tensor]:
        return self._in_meta.empty(self.device)

    def _as_input(self, bufs: List[torch.Tensor]) -> Activation:
        for t, g in zip(bufs, self._in_meta.grads):
            if g:
                t.requires_grad_(True)
        return tuple(bufs) if self._in_meta.is_tuple else bufs[0]

    def _grad_bufs(self) -> List[torch.Tensor]:
        return [torch.empty(s, dtype=d, device=self.device)
                for s, d, g in zip(self._out_meta.shapes, self._out_meta.dtypes, self._out_meta.grads) if g]

    def _input_grads(self, x: Activation) -> List[torch.Tensor]:
        out = []
        for t, g in zip(_flatten(x), self._in_meta.grads):
            if g:
                out.append(t.grad if t.grad is not None else torch.zeros_like(t))
        return out

    # ------------------------------------------------------------------ steps
    def _forward_step(self, x: Optional[Activation], data_iter: Optional[Iterator[Any]]
                      ) -> Tuple[Optional[Activation], Activation, Any]:
        labels = None
        if self.is_first or self.is_last:
            inputs, labels = self._next_batch(data_iter)
            if self.is_first:
                x = inputs
        y = self.module(x)
        if self.is_last:
            if self.module.loss_fn is not None:
                y = self.module.loss_fn(y, labels)
            if not isinstance(y, torch.Tensor) or y.numel() != 1:
                raise ValueError("the last pipeline stage must produce a scalar loss "
                                 "(set PipelineModule(loss_fn=...))")
        return x, y, labels

    def _backward_step(self, x: Optional[Activation], y: Activation,
                       grads: Optional[List[torch.Tensor]]) -> List[torch.Tensor]:
        if self.is_last:
            loss = y / self.micro_batches
            if self._static_scale is not None:
                loss = loss * self._static_scale.to(loss.dtype)
            loss.backward()
        else:
            outs = [t for t, g in zip(_flatten(y), self._out_meta.grads) if g]
            torch.autograd.backward(outs, grads)
        if self.is_first:
            return []
        return self._input_grads(x)

    def _sync_grads_before(self, micro: int, tied: bool) -> None:
        # data-parallel reduction rides the last micro-batch's backward, unless tied weights
        # must be summed over their stages first (then everything reduces after backward)
        self._set_sync(micro == self.micro_batches - 1 and not tied)

    # ------------------------------------------------------------------ schedules
    def train_batch(self, data_iter: Optional[Iterator[Any]] = None) -> torch.Tensor:
        """One optimizer step over ``gradient_accumulation_steps`` micro-batches (1F1B)."""
        if not torch.is_grad_enabled():
            raise RuntimeError("train_batch() requires gradients enabled")
        self.module.train()
        M, S, s = self.micro_batches, self.num_stages, self.stage_id
        tied = bool(self._tie_groups)
        warmup = min(S - s - 1, M)
        remaining = M - warmup
        pending: List[Tuple[Any, Any]] = []
        losses: List[torch.Tensor] = []
        fwd_done = 0
        bwd_done = 0

        def fwd(x_in: Optional[Activation]) -> Activation:
            nonlocal fwd_done
            x, y, _ = self._forward_step(x_in, data_iter)
            if self.is_last:
                losses.append(y.detach().float())
            pending.append((x, y))
            fwd_done += 1
            return y

        def bwd(grads: Optional[List[torch.Tensor]]) -> List[torch.Tensor]:
            nonlocal bwd_done
            x, y = pending.pop(0)
            self._sync_grads_before(bwd_done, tied)
            g = self._backward_step(x, y, grads)
            bwd_done += 1
            return g

        def recv_forward() -> Optional[Activation]:
            if self.is_first:
                return None
            if fwd_done == 0:
                self._recv_meta()
            bufs = self._new_input()
            self._p2p.run([], [(b, self.prev_rank) for b in bufs])
            return self._as_input(bufs)

        def send_forward(y: Activation) -> None:
            if self.is_last:
                return
            if fwd_done == 1:
                self._send_meta(y)
            self._p2p.run([(t, self.next_rank) for t in self._act_tensors(y)], [])

        for _ in range(warmup):
            x = recv_forward()
            send_forward(fwd(x))
        x = recv_forward() if remaining > 0 else None
        for i in range(remaining):
            y = fwd(x)
            # send activations forward, receive the matching output gradient (fused)
            grads: Optional[List[torch.Tensor]] = None
            if not self.is_last:
                if fwd_done == 1:
                    self._send_meta(y)
                grads = self._grad_bufs()
                self._p2p.run([(t, self.next_rank) for t in self._act_tensors(y)],
                              [(b, self.next_rank) for b in grads])
            in_grads = bwd(grads)
            last = i == remaining - 1
            sends = [(t, self.prev_rank) for t in in_grads] if not self.is_first else []
            if last:
                self._p2p.run(sends, [])
            else:
                # send input gradients back, receive the next micro-batch's activations (fused)
                bufs = self._new_input() if not self.is_first else []
                self._p2p.run(sends, [(b, self.prev_rank) for b in bufs])
                x = self._as_input(bufs) if not self.is_first else None
        for _ in range(warmup):
            grads = self._grad_bufs()
            self._p2p.run([], [(b, self.next_rank) for b in grads])
            in_grads = bwd(grads)
            if not self.is_first:
                self._p2p.run([(t, self.prev_rank) for t in in_grads], [])
        assert fwd_done == M and bwd_done == M and not pending

        if tied:
            self._reduce_tied_grads()
        self._set_sync(True)
        self._take_model_step(None)
        self.micro_steps += M
        self.global_samples += self.config.micro_batch * M * self.grid.data_parallel_size
        self.agg_train_loss = self._aggregate_loss(losses)
        return self.agg_train_loss

    @torch.no_grad()
    def eval_batch(self, data_iter: Optional[Iterator[Any]] = None, compute_loss: bool = True,
                   reduce_output: Optional[str] = "avg", num_micro_batches: Optional[int] = None
                   ) -> torch.Tensor:
        """Forward-only pipeline over ``num_micro_batches`` (default: accumulation steps)
        micro-batches; returns the loss averaged over micro-batches and data-parallel ranks, on
        every stage."""
        if not compute_loss:
            raise NotImplementedError("eval_batch(compute_loss=False) is not supported")
        self.module.eval()
        M = int(num_micro_batches or self.micro_batches)
        losses: List[torch.Tensor] = []
        for i in range(M):
            x: Optional[Activation] = None
            if not self.is_first:
                if i == 0:
                    self._recv_meta()
                bufs = self._new_input()
                self._p2p.run([], [(b, self.prev_rank) for b in bufs])
                x = tuple(bufs) if self._in_meta.is_tuple else bufs[0]
            _, y, _ = self._forward_step(x, data_iter)
            if self.is_last:
                losses.append(y.float())
            else:
                if i == 0:
                    self._send_meta(y)
                self._p2p.run([(t, self.next_rank) for t in self._act_tensors(y)], [])
        self.module.train()
        return self._aggregate_loss(losses, reduce_dp=reduce_output is not None)

    def _aggregate_loss(self, losses: List[torch.Tensor], reduce_dp: bool = True) -> torch.Tensor:
        if self.is_last:
            out = torch.stack(losses).mean().reshape(1) if losses else \
                torch.zeros(1, device=self.device)
            if reduce_dp and self.grid.data_parallel_size > 1:
                self._allreduce(out, self.grid.dp_group)
                out /= self.grid.data_parallel_size
        else:
            out = torch.zeros(1, dtype=torch.float32, device=self.device)
        if self.num_stages > 1:
            self._bcast(out, self.grid.stage_to_global(self.num_stages - 1), self.grid.pp_group)
        return out.reshape(())

    # ------------------------------------------------------------------ guards
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        if self.num_stages > 1:
            raise RuntimeError("a pipeline-parallel engine is driven by train_batch()/eval_batch()")
        return self.module(*args, **kwargs)

    def backward(self, *args: Any, **kwargs: Any) -> Any:
        raise RuntimeError("a pipeline-parallel engine is driven by train_batch()/eval_batch()")

    def step(self, *args: Any, **kwargs: Any) -> None:
        raise RuntimeError("a pipeline-parallel engine is driven by train_batch()/eval_batch()")

    def is_gradient_accumulation_boundary(self) -> bool:
        return True

    # ------------------------------------------------------------------ checkpoint
    def _mp_tag(self, sep: str) -> str:
        """File-name part for the TP rank (DeepSpeed's ``-model_XX``); empty without TP."""
        return f"{sep}{self.grid.model_parallel_id:02d}" if self.grid.model_parallel_size > 1 else ""

    def save_checkpoint(self, save_dir: Union[str, pathlib.Path], tag: Optional[str] = None,
                        client_state: Optional[Dict[str, Any]] = None,
                        save_latest: bool = True) -> bool:
        """``<dir>/<tag>/layer_XX-model_states.pt`` per layer (data-parallel rank 0 of the owning
        stage), ``mp_rank_00_model_states.pt`` (global rank 0: counters, scheduler, client state)
        and ``pipe_stage_XX_dp_YY_optim_states.pt`` (optimizer, per stage and, for ZeRO, per
        data-parallel rank)."""
        tag = tag or f"global_step{self.global_steps}"
        d = pathlib.Path(save_dir) / str(tag)
        d.mkdir(parents=True, exist_ok=True)
        dp = self.grid.data_parallel_id
        wait = getattr(self.optimizer, "wait_params", None)
        if wait is not None:  # ZeRO-1/2: parameter all-gathers may still be in flight
            wait()
        if dp == 0:
            for idx, sd in self.module.layer_state_dicts().items():
                torch.save(sd, d / f"layer_{idx:02d}{self._mp_tag('-model_')}-model_states.pt")
        if self.config.zero_stage >= 1 or dp == 0:
            torch.save({"optimizer_state_dict": self.optimizer.state_dict(),
                        "parts": list(self.module.parts),
                        "dp_world_size": self.grid.data_parallel_size},
                       d / f"pipe_stage_{self.stage_id:02d}_dp_{dp:02d}{self._mp_tag('_mp_')}_optim_states.pt")
        if self.grid.global_rank == 0:
            torch.save({
                "module": None,
                "lr_scheduler": self.lr_scheduler.state_dict() if self.lr_scheduler is not None else None,
                "global_steps": self.global_steps, "global_samples": self.global_samples,
                "micro_steps": self.micro_steps, "skipped_steps": self.skipped_steps,
                "num_stages": self.num_stages, "parts": list(self.module.parts),
                "dp_world_size": self.grid.data_parallel_size,
                "zero_stage": self.config.zero_stage, "client_state": client_state or {},
            }, d / "mp_rank_00_model_states.pt")
            if save_latest:
                (pathlib.Path(save_dir) / "latest").write_text(str(tag))
        return True

    def load_checkpoint(self, load_dir: Union[str, pathlib.Path], tag: Optional[str] = None,
                        load_module_strict: bool = True, load_optimizer_states: bool = True,
                        load_lr_scheduler_states: bool = True
                        ) -> Tuple[Optional[str], Optional[Dict[str, Any]]]:
        load_dir = pathlib.Path(load_dir)
        if tag is None:
            latest = load_dir / "latest"
            if not latest.exists():
                logger.warning(f"no 'latest' file under {load_dir}; nothing loaded")
                return None, None
            tag = latest.read_text().strip()
        d = load_dir / str(tag)
        state = torch.load(d / "mp_rank_00_model_states.pt", map_location="cpu", weights_only=True)
        start, stop = self.module.stage_layers()
        layers = {}
        for idx in range(start, stop):
            p = d / f"layer_{idx:02d}{self._mp_tag('-model_')}-model_states.pt"
            if p.exists():
                layers[idx] = torch.load(p, map_location="cpu", weights_only=True)
        self.module.load_layer_state_dicts(layers, strict=load_module_strict)
        self.global_steps = int(state.get("global_steps", 0))
        self.global_samples = int(state.get("global_samples", 0))
        self.micro_steps = int(state.get("micro_steps", 0))
        self.skipped_steps = int(state.get("skipped_steps", 0))
        if load_lr_scheduler_states and self.lr_scheduler is not None and state.get("lr_scheduler"):
            self.lr_scheduler.load_state_dict(state["lr_scheduler"])
        same_layout = list(state.get("parts", [])) == list(self.module.parts) and \
            int(state.get("dp_world_size", -1)) == self.grid.data_parallel_size
        dp = self.grid.data_parallel_id if self.config.zero_stage >= 1 else 0
        opt_path = d / f"pipe_stage_{self.stage_id:02d}_dp_{dp:02d}{self._mp_tag('_mp_')}_optim_states.pt"
        if load_optimizer_states and same_layout and opt_path.exists():
            osd = torch.load(opt_path, map_location="cpu", weights_only=True)["optimizer_state_dict"]
            from determined_clone_amd.parallel import zero

            if isinstance(self.optimizer, zero.ZeroShardMixin):
                self.optimizer.load_shard_state_dicts([osd])
            else:
                self.optimizer.load_state_dict(osd)
                if not any("master_param" in s for s in osd["state"].values()):
                    self.optimizer.sync_master_from_model()
        else:
            if load_optimizer_states and not same_layout:
                logger.warning("pipeline partition or data-parallel size changed since the "
                               "checkpoint: model weights loaded, optimizer state reset")
            self.optimizer.sync_master_from_model()
        return str(d), state.get("client_state", {})
