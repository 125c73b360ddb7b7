"""Tensor-parallel GPT-2 / GPT-NeoX (Megatron layout) on ``parallel/tensor.py``.

The reference's GPT-NeoX trial trains with ``model_parallel_size: 2``
(`examples/deepspeed/gpt_neox/zero1.yaml:15-16`, gpt-neox's Megatron mpu). Same math as
:class:`~determined_clone_amd.models.gpt2.GPT`, sharded over a TP group of ``tp`` ranks:

* attention heads are split: the fused QKV projection is column-parallel over whole heads (each
  rank owns the q, k and v rows of its ``n_head / tp`` heads, so the local [B, S, 3, H/tp, D]
  output feeds the MFMA flash-attention kernel unchanged) and the output projection is
  row-parallel -> one all-reduce per attention block;
* the MLP up-projection is column-parallel (bias + GELU fused on the local columns), the
  down-projection row-parallel -> one all-reduce per MLP;
* token embedding and the tied LM head are vocab-parallel; the loss is the vocab-parallel
  cross-entropy, so the [tokens, vocab] logits are never gathered;
* LayerNorms, position embeddings and row-parallel biases are replicated (identical gradients on
  every TP rank; :func:`~determined_clone_amd.parallel.tensor.tp_norm_setup` counts them once).

``TPGPT.load_from(full)`` copies a dense model's weights into the shards (parity tests, and
converting dense checkpoints); ``full_state_dict()`` gathers them back.
"""
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.models.gpt2 import GPT, FusedLayerNorm, GPTConfig, _init_like_gpt
from determined_clone_amd.ops import transformer as T
from determined_clone_amd.parallel import tensor as tp


class TPAttention(nn.Module):
    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__()
        self.cfg, self.group = cfg, group
        n = tp._size(group)
        if cfg.n_head % n:
            raise ValueError(f"n_head {cfg.n_head} not divisible by TP size {n}")
        self.local_heads = cfg.n_head // n
        E = cfg.d_model
        self.qkv = tp.ColumnParallelLinear(E, 3 * E, group)
        self.proj = tp.RowParallelLinear(E, E, group)
        self.rot = 0
        if cfg.pos_emb == "rotary":
            rot = int(cfg.head_dim * cfg.rotary_pct)
            self.rot = rot - rot % 2

    def qkv_rows(self) -> torch.Tensor:
        """Rows of the dense [3E, E] QKV weight this rank owns: its heads' q, k and v rows."""
        E, D = self.cfg.d_model, self.cfg.head_dim
        h0 = tp._rank(self.group) * self.local_heads
        span = torch.arange(h0 * D, (h0 + self.local_heads) * D)
        return torch.cat([j * E + span for j in range(3)])

    def forward(self, x: torch.Tensor, rope_cache: Any = None) -> torch.Tensor:
        B, S, _ = x.shape
        H, D = self.local_heads, self.cfg.head_dim
        qkv = self.qkv(x).view(B, S, 3, H, D)
        if self.rot:
            q, k, v = qkv.unbind(2)
            cos, sin = rope_cache
            o = T.flash_attention(T.rope(q, cos, sin, self.rot), T.rope(k, cos, sin, self.rot), v,
                                  causal=True)
        else:
            o = T.flash_attention_qkvpacked(qkv, causal=True)
        if self.cfg.dropout and self.training:
            o = F.dropout(o, self.cfg.dropout)
        return self.proj(o.reshape(B, S, H * D))


class TPMLP(nn.Module):
    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__()
        E = cfg.d_model
        self.fc = tp.ColumnParallelLinear(E, cfg.mlp_ratio * E, group)
        self.proj = tp.RowParallelLinear(cfg.mlp_ratio * E, E, group)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.proj(T.bias_gelu(self.fc(x, fuse_bias=False), self.fc.bias))


class TPBlock(nn.Module):
    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__()
        if cfg.dropout and tp._size(group) > 1:
            # dropout on the replicated residual stream must draw the same mask on every TP rank
            # (Megatron's model-parallel RNG tracker); not provided here
            raise NotImplementedError("dropout > 0 with tensor parallelism is not supported")
        self.ln1 = FusedLayerNorm(cfg.d_model, cfg.ln_eps)
        self.attn = TPAttention(cfg, group)
        self.ln2 = FusedLayerNorm(cfg.d_model, cfg.ln_eps)
        self.mlp = TPMLP(cfg, group)
        self.dropout = cfg.dropout

    def forward(self, resid: torch.Tensor, delta: Optional[torch.Tensor], rope_cache: Any = None):
        if delta is None:
            h = self.ln1(resid)
        else:
            h, resid = self.ln1(resid, residual=delta)
        a = self.attn(h, rope_cache)
        h, resid = self.ln2(resid, residual=a)
        m = self.mlp(h)
        if self.dropout and self.training:
            m = F.dropout(m, self.dropout)
        return resid, m


class TPGPT(nn.Module):
    """GPT sharded over the TP ``group`` (``None`` or size 1 = dense math on one rank)."""

    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__()
        if not cfg.tie_embeddings:
            raise ValueError("TPGPT uses the tied vocab-parallel embedding as its LM head")
        self.cfg, self.group = cfg, group
        V, E = cfg.padded_vocab, cfg.d_model
        self.wte = tp.VocabParallelEmbedding(V, E, group)
        self.wpe = nn.Embedding(cfg.max_seq_len, E) if cfg.pos_emb == "learned" else None
        self.blocks = nn.ModuleList([TPBlock(cfg, group) for _ in range(cfg.n_layer)])
        self.ln_f = FusedLayerNorm(E, cfg.ln_eps)
        if cfg.pos_emb == "rotary":
            cos, sin = T.rope_tables(cfg.max_seq_len, self.blocks[0].attn.rot, cfg.rotary_base)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
        _init_like_gpt(self, cfg)
        tp_reinit_(self, cfg, group)

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None):
        B, S = idx.shape
        x = self.wte(idx)
        if self.wpe is not None:
            x = x + self.wpe.weight[:S].unsqueeze(0)
        rope = (self.rope_cos, self.rope_sin) if self.cfg.pos_emb == "rotary" else None
        resid, delta = x, None
        for blk in self.blocks:
            resid, delta = blk(resid, delta, rope)
        h, _ = self.ln_f(resid, residual=delta)
        logits = F.linear(tp.copy_to_tp(h, self.group), self.wte.weight)  # vocab shard
        if targets is None:
            return logits
        loss = tp.vocab_parallel_cross_entropy(logits, targets, self.group, self.wte.start)
        return logits, loss

    # ------------------------------------------------------------------ dense <-> sharded
    @torch.no_grad()
    def load_from(self, full: GPT) -> "TPGPT":
        """Copy a dense :class:`GPT`'s weights into this rank's shards."""
        self.wte.load_full(full.wte.weight)
        if self.wpe is not None:
            self.wpe.weight.copy_(full.wpe.weight)
        self.ln_f.load_state_dict(full.ln_f.state_dict())
        for b, fb in zip(self.blocks, full.blocks):
            b.ln1.load_state_dict(fb.ln1.state_dict())
            b.ln2.load_state_dict(fb.ln2.state_dict())
            b.attn.qkv.load_full(fb.attn.qkv.weight, fb.attn.qkv.bias, rows=b.attn.qkv_rows())
            b.attn.proj.load_full(fb.attn.proj.weight, fb.attn.proj.bias)
            b.mlp.fc.load_full(fb.mlp.fc.weight, fb.mlp.fc.bias)
            b.mlp.proj.load_full(fb.mlp.proj.weight, fb.mlp.proj.bias)
        return self

    def full_state_dict(self) -> Dict[str, torch.Tensor]:
        """The dense model's state dict, gathered over the TP group (every TP rank must call)."""
        n = tp._size(self.group)

        def gather(t: torch.Tensor, dim: int) -> torch.Tensor:
            if n == 1:
                return t.detach().clone()
            parts = [torch.empty_like(t) for _ in range(n)]
            dist.all_gather(parts, t.detach().contiguous(), group=self.group)
            return torch.cat(parts, dim=dim)

        out: Dict[str, torch.Tensor] = {"wte.weight": gather(self.wte.weight, 0)}
        if self.wpe is not None:
            out["wpe.weight"] = self.wpe.weight.detach().clone()
        for k, v in self.ln_f.state_dict().items():
            out[f"ln_f.{k}"] = v.clone()
        E, D = self.cfg.d_model, self.cfg.head_dim
        for i, b in enumerate(self.blocks):
            p = f"blocks.{i}."
            for ln in ("ln1", "ln2"):
                for k, v in getattr(b, ln).state_dict().items():
                    out[p + f"{ln}.{k}"] = v.clone()
            # QKV: each rank holds [q_h; k_h; v_h] of its heads -> reorder to [q; k; v]
            Hl = b.attn.local_heads
            for name, t in (("weight", b.attn.qkv.weight), ("bias", b.attn.qkv.bias)):
                g = gather(t, 0).reshape(n, 3, Hl * D, *t.shape[1:])
                out[p + f"attn.qkv.{name}"] = g.transpose(0, 1).reshape(3 * E, *t.shape[1:])
            out[p + "attn.proj.weight"] = gather(b.attn.proj.weight, 1)
            out[p + "attn.proj.bias"] = b.attn.proj.bias.detach().clone()
            out[p + "mlp.fc.weight"] = gather(b.mlp.fc.weight, 0)
            out[p + "mlp.fc.bias"] = gather(b.mlp.fc.bias, 0)
            out[p + "mlp.proj.weight"] = gather(b.mlp.proj.weight, 1)
            out[p + "mlp.proj.bias"] = b.mlp.proj.bias.detach().clone()
        return out


def tp_reinit_(module: nn.Module, cfg: GPTConfig, group: Any) -> None:
    """Re-draw the TP-sharded parameters from a per-TP-rank generator (Megatron's model-parallel
    RNG): with one global seed every rank would otherwise draw identical shards, i.e. duplicated
    heads / MLP columns. Replicated parameters keep the global RNG's (identical) values."""
    if tp._size(group) <= 1 or any(p.is_meta for p in module.parameters()):
        return  # (meta: PipelineModule sizing its partition without materialising layers)
    import math

    base = int(torch.randint(0, 2 ** 31 - 1, (1,), device="cpu").item())  # same seed -> same on every rank
    gen = torch.Generator().manual_seed(base + 7919 * (tp._rank(group) + 1))
    proj_std = cfg.init_std / math.sqrt(2 * cfg.n_layer)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if not getattr(p, "tensor_model_parallel", False) or p.dim() < 2:
                continue
            std = proj_std if name.endswith("proj.weight") else cfg.init_std
            p.copy_(torch.randn(p.shape, generator=gen) * std)


# ---------------------------------------------------------------------------------- pipe x tensor
class EmbeddingPipeTP(nn.Module):
    """Vocab-parallel token (+ replicated learned position) embedding for a pipeline stage."""

    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__()
        self.cfg = cfg
        self.wte = tp.VocabParallelEmbedding(cfg.padded_vocab, cfg.d_model, group)
        self.wpe = nn.Embedding(cfg.max_seq_len, cfg.d_model) if cfg.pos_emb == "learned" else None
        _init_like_gpt(self, cfg)
        tp_reinit_(self, cfg, group)

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        x = self.wte(idx)
        if self.wpe is not None:
            x = x + self.wpe.weight[:idx.shape[1]].unsqueeze(0)
        return x


class BlockPipeTP(TPBlock):
    """Tensor-parallel block on a pipeline activation (residual, or (residual, pending delta))."""

    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        super().__init__(cfg, group)
        self.rotary = cfg.pos_emb == "rotary"
        if self.rotary:
            cos, sin = T.rope_tables(cfg.max_seq_len, self.attn.rot, cfg.rotary_base)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
        _init_like_gpt(self, cfg)
        tp_reinit_(self, cfg, group)

    def forward(self, x):  # type: ignore[override]
        resid, delta = (x, None) if isinstance(x, torch.Tensor) else x
        rope = (self.rope_cos, self.rope_sin) if self.rotary else None
        return super().forward(resid, delta, rope)


def _tied_head_tp(module: nn.Module, h: torch.Tensor) -> torch.Tensor:
    return F.linear(tp.copy_to_tp(h, module.wte.group), module.wte.weight)


class PipelineLossTP:
    """Vocab-parallel cross-entropy on the last stage (the logits are this rank's vocab shard)."""

    def __init__(self, cfg: GPTConfig, group: Any) -> None:
        self.group = group
        self.start = tp._rank(group) * (cfg.padded_vocab // tp._size(group))

    def __call__(self, logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        return tp.vocab_parallel_cross_entropy(logits, targets, self.group, self.start)


def pipeline_specs_tp(cfg: GPTConfig, group: Any) -> list:
    """:func:`~determined_clone_amd.models.gpt2.pipeline_specs` with tensor-parallel layers: the
    reference gpt_neox layout with pipe_parallel_size x model_parallel_size (zero1.yaml: 2 x 2).
    Use with ``PipelineModule(..., grid=ModelParallelGrid(M, P), loss_fn=PipelineLossTP(cfg,
    grid.mp_group))``."""
    from determined_clone_amd.models.gpt2 import FinalNormPipe
    from determined_clone_amd.parallel.pipeline import LayerSpec, TiedLayerSpec

    if not cfg.tie_embeddings:
        raise ValueError("the tensor-parallel pipeline uses the tied vocab-parallel embedding as LM head")
    embed = TiedLayerSpec("embed", EmbeddingPipeTP, cfg, group, tied_weight_attr="wte.weight")
    head = TiedLayerSpec("embed", EmbeddingPipeTP, cfg, group, forward_fn=_tied_head_tp,
                         tied_weight_attr="wte.weight")
    return [embed] + [LayerSpec(BlockPipeTP, cfg, group) for _ in range(cfg.n_layer)] + \
        [LayerSpec(FinalNormPipe, cfg), head]


@torch.no_grad()
def load_pipeline_from(pipe_module: nn.Module, full: GPT) -> None:
    """Copy a dense :class:`GPT` into the local stage's layers of a
    :func:`pipeline_specs_tp` PipelineModule (layer 0 embedding, 1..L blocks, L+1 final norm,
    L+2 tied head)."""
    L = full.cfg.n_layer
    for idx, mod in pipe_module._layer_modules.items():
        if isinstance(mod, EmbeddingPipeTP):
            mod.wte.load_full(full.wte.weight)
            if mod.wpe is not None:
                mod.wpe.weight.copy_(full.wpe.weight)
        elif isinstance(mod, TPBlock):
            fb = full.blocks[idx - 1]
            mod.ln1.load_state_dict(fb.ln1.state_dict())
            mod.ln2.load_state_dict(fb.ln2.state_dict())
            mod.attn.qkv.load_full(fb.attn.qkv.weight, fb.attn.qkv.bias, rows=mod.attn.qkv_rows())
            mod.attn.proj.load_full(fb.attn.proj.weight, fb.attn.proj.bias)
            mod.mlp.fc.load_full(fb.mlp.fc.weight, fb.mlp.fc.bias)
            mod.mlp.proj.load_full(fb.mlp.proj.weight, fb.mlp.proj.bias)
        elif idx == L + 1:
            mod.ln_f.load_state_dict(full.ln_f.state_dict())
