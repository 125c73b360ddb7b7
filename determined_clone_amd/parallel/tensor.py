"""Tensor (model / slice) parallelism: Megatron-style sharded layers over RCCL.

The reference's GPT-NeoX DeepSpeedTrial runs ``model_parallel_size: 2`` (with
``pipe_parallel_size: 2``, `examples/deepspeed/gpt_neox/zero1.yaml:15-16`) through the gpt-neox /
Megatron ``mpu``; its harness only sees the mpu's data-parallel rank and size
(`harness/determined/pytorch/deepspeed/_mpu.py`). Here the layers themselves:

* :class:`ModelParallelGrid` -- ``pipe x data x model`` process grid (model-parallel ranks are
  adjacent, so a TP group sits on neighbouring GPUs: on one MI355X node that keeps the per-layer
  all-reduces on direct xGMI links), DeepSpeed / Megatron accessors for ``make_deepspeed_mpu``;
* :class:`ColumnParallelLinear` (output features sharded; input gradient all-reduced),
  :class:`RowParallelLinear` (input features sharded; output all-reduced, bias added once),
  :class:`VocabParallelEmbedding`, :func:`vocab_parallel_cross_entropy` (softmax statistics
  all-reduced, the [tokens, vocab] logits never gathered);
* :func:`mark_tensor_parallel` / :func:`tp_norm_setup` -- which parameters are sharded, so the
  global gradient norm counts replicated parameters once (optimizer ``norm_group`` /
  ``norm_exclude``).

The local GEMMs are the same fused MFMA paths as the dense model (``ops.transformer.linear``):
splitting heads / MLP columns keeps every per-rank GEMM a plain row-major GEMM, and one
all-reduce per attention block and per MLP (forward and backward) is the whole TP traffic.
"""
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import transformer as T


def _size(group: Any) -> int:
    return dist.get_world_size(group) if group is not None and dist.is_initialized() else 1


def _rank(group: Any) -> int:
    return dist.get_rank(group) if group is not None and dist.is_initialized() else 0


# ---------------------------------------------------------------------------------- grid
class ModelParallelGrid:
    """``pipe x data x model`` grid: global rank = (stage * D + d) * M + m. Every rank constructs
    it (group creation is collective)."""

    def __init__(self, model_parallel_size: int = 1, pipe_parallel_size: int = 1) -> None:
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0
        M, P = int(model_parallel_size), int(pipe_parallel_size)
        if M <= 0 or P <= 0 or self.world_size % (M * P):
            raise ValueError(f"world size {self.world_size} is not divisible by model_parallel_size "
                             f"{M} x pipe_parallel_size {P}")
        D = self.world_size // (M * P)
        self.model_parallel_size, self.pipe_parallel_size, self.data_parallel_size = M, P, D
        r = self.global_rank
        self.model_parallel_id = r % M
        self.data_parallel_id = (r // M) % D
        self.stage_id = r // (M * D)
        self.mp_group = self.dp_group = self.pp_group = None

        def rank_of(s: int, d: int, m: int) -> int:
            return (s * D + d) * M + m

        self.rank_of = rank_of
        if not dist.is_initialized() or self.world_size == 1:
            return
        # new_group is collective: every rank creates every group in the same order
        for s in range(P):
            for d in range(D):
                ranks = [rank_of(s, d, m) for m in range(M)]
                g = dist.new_group(ranks)
                if r in ranks:
                    self.mp_group = g
        for s in range(P):
            for m in range(M):
                ranks = [rank_of(s, d, m) for d in range(D)]
                g = dist.new_group(ranks)
                if r in ranks:
                    self.dp_group = g
        for d in range(D):
            for m in range(M):
                ranks = [rank_of(s, d, m) for s in range(P)]
                g = dist.new_group(ranks)
                if r in ranks:
                    self.pp_group = g

    def stage_to_global(self, stage_id: int, data_parallel_id: Optional[int] = None,
                        model_parallel_id: Optional[int] = None) -> int:
        d = self.data_parallel_id if data_parallel_id is None else data_parallel_id
        m = self.model_parallel_id if model_parallel_id is None else model_parallel_id
        return self.rank_of(stage_id, d, m)

    # DeepSpeed / Megatron accessors
    def get_model_parallel_rank(self) -> int:
        return self.model_parallel_id

    def get_model_parallel_world_size(self) -> int:
        return self.model_parallel_size

    def get_model_parallel_group(self) -> Any:
        return self.mp_group

    get_slice_parallel_rank = get_model_parallel_rank
    get_slice_parallel_world_size = get_model_parallel_world_size
    get_slice_parallel_group = get_model_parallel_group
    get_tensor_model_parallel_rank = get_model_parallel_rank
    get_tensor_model_parallel_world_size = get_model_parallel_world_size
    get_tensor_model_parallel_group = get_model_parallel_group

    def get_data_parallel_rank(self) -> int:
        return self.data_parallel_id

    def get_data_parallel_world_size(self) -> int:
        return self.data_parallel_size

    def get_data_parallel_group(self) -> Any:
        return self.dp_group

    def get_pipe_parallel_rank(self) -> int:
        return self.stage_id

    def get_pipe_parallel_world_size(self) -> int:
        return self.pipe_parallel_size

    def get_pipe_parallel_group(self) -> Any:
        return self.pp_group

    get_stage_id = get_pipe_parallel_rank


# ---------------------------------------------------------------------------------- mappings
class _CopyToTP(torch.autograd.Function):
    """Identity forward; all-reduce of the input gradient (the input feeds every shard)."""

    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """All-reduce forward (sum of the shards' partial products); identity backward."""

    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        return g, None


class _GatherFromTP(torch.autograd.Function):
    """All-gather along the last dim forward; keep the own slice backward."""

    @staticmethod
    def forward(ctx, x, group):  # type: ignore[override]
        ctx.group = group
        n = _size(group)
        parts = [torch.empty_like(x) for _ in range(n)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        n, r = _size(ctx.group), _rank(ctx.group)
        return g.chunk(n, dim=-1)[r].contiguous(), None


def copy_to_tp(x: torch.Tensor, group: Any) -> torch.Tensor:
    return _CopyToTP.apply(x, group) if _size(group) > 1 else x


def reduce_from_tp(x: torch.Tensor, group: Any) -> torch.Tensor:
    return _ReduceFromTP.apply(x, group) if _size(group) > 1 else x


def gather_from_tp(x: torch.Tensor, group: Any) -> torch.Tensor:
    return _GatherFromTP.apply(x, group) if _size(group) > 1 else x


def mark_tensor_parallel(p: torch.Tensor) -> torch.Tensor:
    """Tag a parameter as sharded across the TP group (its norm is summed over the group)."""
    p.tensor_model_parallel = True  # type: ignore[attr-defined]
    return p


# ---------------------------------------------------------------------------------- layers
class ColumnParallelLinear(nn.Module):
    """``y = x W^T + b`` with W's output rows split over the TP group: rank r holds rows
    ``[r*out/tp, (r+1)*out/tp)``. ``gather_output`` all-gathers ``y`` (otherwise each rank keeps
    its column block, ready for a :class:`RowParallelLinear`). ``row_index`` optionally gives the
    full-weight rows this rank owns (e.g. q/k/v heads of a fused QKV projection)."""

    def __init__(self, in_features: int, out_features: int, group: Any, bias: bool = True,
                 gather_output: bool = False) -> None:
        super().__init__()
        tp = _size(group)
        if out_features % tp:
            raise ValueError(f"out_features {out_features} not divisible by TP size {tp}")
        self.group, self.gather_output = group, gather_output
        self.in_features, self.out_features = in_features, out_features
        self.weight = mark_tensor_parallel(nn.Parameter(torch.empty(out_features // tp, in_features)))
        self.bias = mark_tensor_parallel(nn.Parameter(torch.zeros(out_features // tp))) if bias else None
        nn.init.normal_(self.weight, 0.0, 0.02)

    def row_index(self) -> torch.Tensor:
        n = self.out_features // _size(self.group)
        return torch.arange(_rank(self.group) * n, (_rank(self.group) + 1) * n)

    @torch.no_grad()
    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
                  rows: Optional[torch.Tensor] = None) -> None:
        rows = self.row_index() if rows is None else rows
        self.weight.copy_(weight[rows.to(weight.device)])
        if self.bias is not None and bias is not None:
            self.bias.copy_(bias[rows.to(bias.device)])

    def forward(self, x: torch.Tensor, fuse_bias: bool = True) -> torch.Tensor:
        x = copy_to_tp(x, self.group)
        y = T.linear(x, self.weight, self.bias if fuse_bias else None)
        return gather_from_tp(y, self.group) if self.gather_output else y


class RowParallelLinear(nn.Module):
    """``y = x W^T + b`` with W's input columns split over the TP group; the input arrives split
    (a :class:`ColumnParallelLinear`'s output); partial products are all-reduced and the bias is
    added once after the reduction."""

    def __init__(self, in_features: int, out_features: int, group: Any, bias: bool = True) -> None:
        super().__init__()
        tp = _size(group)
        if in_features % tp:
            raise ValueError(f"in_features {in_features} not divisible by TP size {tp}")
        self.group = group
        self.in_features, self.out_features = in_features, out_features
        self.weight = mark_tensor_parallel(nn.Parameter(torch.empty(out_features, in_features // tp)))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None  # replicated
        nn.init.normal_(self.weight, 0.0, 0.02)

    def col_index(self) -> torch.Tensor:
        n = self.in_features // _size(self.group)
        return torch.arange(_rank(self.group) * n, (_rank(self.group) + 1) * n)

    @torch.no_grad()
    def load_full(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> None:
        self.weight.copy_(weight[:, self.col_index().to(weight.device)])
        if self.bias is not None and bias is not None:
            self.bias.copy_(bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = reduce_from_tp(T.linear(x, self.weight), self.group)
        return y + self.bias.to(y.dtype) if self.bias is not None else y


class VocabParallelEmbedding(nn.Module):
    """Embedding table split by vocabulary rows; out-of-shard tokens look up zeros and the shards'
    rows are summed by one all-reduce. Its weight doubles as the vocab-parallel LM head."""

    def __init__(self, num_embeddings: int, embedding_dim: int, group: Any) -> None:
        super().__init__()
        tp = _size(group)
        if num_embeddings % tp:
            raise ValueError(f"vocab {num_embeddings} not divisible by TP size {tp}")
        self.group = group
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.per = num_embeddings // tp
        self.start = _rank(group) * self.per
        self.weight = mark_tensor_parallel(nn.Parameter(torch.empty(self.per, embedding_dim)))
        nn.init.normal_(self.weight, 0.0, 0.02)

    @torch.no_grad()
    def load_full(self, weight: torch.Tensor) -> None:
        self.weight.copy_(weight[self.start:self.start + self.per])

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        if _size(self.group) == 1:
            return F.embedding(idx, self.weight)
        local = idx - self.start
        outside = (local < 0) | (local >= self.per)
        out = F.embedding(local.masked_fill(outside, 0), self.weight)
        out = out.masked_fill(outside.unsqueeze(-1), 0)
        return reduce_from_tp(out, self.group)


class _VocabParallelCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, group, start, ignore_index):  # type: ignore[override]
        x = logits.float()
        m = x.max(dim=-1).values
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        x = x - m.unsqueeze(-1)
        ex = x.exp()
        sumexp = ex.sum(dim=-1)
        dist.all_reduce(sumexp, group=group)
        V = x.shape[-1]
        local = target - start
        valid = target != ignore_index
        mine = valid & (local >= 0) & (local < V)
        li = local.clamp(0, V - 1)
        tlogit = torch.where(mine, x.gather(-1, li.unsqueeze(-1)).squeeze(-1), torch.zeros_like(m))
        dist.all_reduce(tlogit, group=group)
        loss = torch.where(valid, sumexp.log() - tlogit, torch.zeros_like(m))
        n = valid.sum().clamp_min(1)
        ctx.save_for_backward(ex, sumexp, li, mine, valid, n)
        ctx.dtype = logits.dtype
        return loss.sum() / n

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        ex, sumexp, li, mine, valid, n = ctx.saved_tensors
        p = ex / sumexp.unsqueeze(-1)
        p.scatter_add_(-1, li.unsqueeze(-1), -mine.to(p.dtype).unsqueeze(-1))
        p = p * (valid.to(p.dtype) * (g / n)).unsqueeze(-1)
        return p.to(ctx.dtype), None, None, None, None


def vocab_parallel_cross_entropy(logits: torch.Tensor, target: torch.Tensor, group: Any,
                                 vocab_start: int, ignore_index: int = -100) -> torch.Tensor:
    """Mean token cross-entropy of vocab-sharded ``logits`` [..., V/tp] (rank's vocab range starts
    at ``vocab_start``); softmax statistics are all-reduced, the full logits never exist."""
    if _size(group) == 1:
        return T.cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1),
                               ignore_index=ignore_index)
    return _VocabParallelCE.apply(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), group,
                                  vocab_start, ignore_index)


# ---------------------------------------------------------------------------------- grad norm
def replicated_params(params: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    return [p for p in params if not getattr(p, "tensor_model_parallel", False)]


def tp_norm_setup(optimizer: Any, params: Sequence[torch.Tensor], group: Any) -> None:
    """Make ``optimizer``'s clip norm the norm of the whole (unsharded) model: the squared norm is
    also summed over the TP group, and replicated parameters (LayerNorms, row-parallel biases,
    position embeddings) are counted only on TP rank 0."""
    if _size(group) <= 1:
        return
    optimizer.norm_group = group
    if _rank(group) != 0:
        optimizer.norm_exclude = list(optimizer.norm_exclude) + replicated_params(params)
