"""GPT-2 / GPT-NeoX-style decoder-only transformer built on the MI355X transformer ops.

Stands in for the GPT-NeoX model the reference's DeepSpeedTrial example trains
(reference: `examples/deepspeed/gpt_neox/gpt2_trial.py`, which builds Megatron/NeoX GPT-2 with
DeepSpeed; BASELINE config "GPT-2-medium DeepSpeedTrial ZeRO-2").

MI355X layout decisions:
* pre-LN blocks where each residual add is fused into the NEXT LayerNorm
  (``ops.transformer.layer_norm(x, residual=delta)`` returns ``(LN(x + delta), x + delta)`` in one
  HBM pass), so a block costs 2 fused add+LN kernels instead of 2 adds + 2 LNs;
* the fused QKV projection output [B, S, 3, H, Dh] is consumed by the MFMA flash-attention kernel
  through strided views (no q/k/v copies, no [S, S] score matrix);
* MLP up-projection runs without bias in hipBLASLt and the bias + tanh-GELU are one fused kernel;
* GEMM weights are bf16; LayerNorm affine parameters stay fp32 (they are read by the LN kernels as
  fp32 and keep their own flat fp32 buffer in the optimizer);
* position encoding: learned absolute (GPT-2) or rotary on the first ``rotary_pct`` of each head
  (GPT-NeoX, rotate-half convention, fused RoPE kernel).
"""
import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import transformer as T


@dataclass
class GPTConfig:
    vocab_size: int = 50257
    n_layer: int = 24
    n_head: int = 16
    d_model: int = 1024
    max_seq_len: int = 1024
    mlp_ratio: int = 4
    pos_emb: str = "learned"  # "learned" (GPT-2) | "rotary" (GPT-NeoX)
    rotary_pct: float = 0.25
    rotary_base: float = 10000.0
    ln_eps: float = 1e-5
    tie_embeddings: bool = True
    dropout: float = 0.0
    init_std: float = 0.02
    pad_vocab_multiple: int = 128
    extra: Dict = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_head

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return (self.vocab_size + m - 1) // m * m


PRESETS = {
    "gpt2-small": dict(n_layer=12, n_head=12, d_model=768),
    "gpt2-medium": dict(n_layer=24, n_head=16, d_model=1024),
    "gpt2-large": dict(n_layer=36, n_head=20, d_model=1280),
    "gpt2-xl": dict(n_layer=48, n_head=25, d_model=1600),
    "neox-125m": dict(n_layer=12, n_head=12, d_model=768, pos_emb="rotary"),
    "neox-350m": dict(n_layer=24, n_head=16, d_model=1024, pos_emb="rotary"),
    "tiny": dict(n_layer=2, n_head=2, d_model=128, vocab_size=512, max_seq_len=128),
}


def config_for(name: str, **overrides) -> GPTConfig:
    kw = dict(PRESETS[name])
    kw.update(overrides)
    return GPTConfig(**kw)


class FusedLayerNorm(nn.Module):
    """LayerNorm whose forward optionally fuses the preceding residual add."""

    keep_fp32 = True  # engines keep these parameters fp32 when casting the model to bf16

    def __init__(self, dim: int, eps: float = 1e-5) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))
        self.eps = eps

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None):
        return T.layer_norm(x, self.weight, self.bias, self.eps, residual=residual)


class Attention(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.cfg = cfg
        E = cfg.d_model
        self.qkv = nn.Linear(E, 3 * E)
        self.proj = nn.Linear(E, E)
        self.rot = 0
        if cfg.pos_emb == "rotary":
            rot = int(cfg.head_dim * cfg.rotary_pct)
            self.rot = rot - rot % 2
        if cfg.head_dim not in (64, 128):
            raise ValueError("head_dim must be 64 or 128 for the MFMA attention kernel")

    def forward(self, x: torch.Tensor, rope_cache=None) -> torch.Tensor:
        B, S, E = x.shape
        H, D = self.cfg.n_head, self.cfg.head_dim
        qkv = T.linear(x, self.qkv.weight, self.qkv.bias).view(B, S, 3, H, D)
        if self.rot:
            q, k, v = qkv.unbind(2)
            cos, sin = rope_cache
            q = T.rope(q, cos, sin, self.rot)
            k = T.rope(k, cos, sin, self.rot)
            o = T.flash_attention(q, k, v, causal=True)
        else:
            o = T.flash_attention_qkvpacked(qkv, causal=True)
        if self.cfg.dropout and self.training:
            o = F.dropout(o, self.cfg.dropout)
        return T.linear(o.reshape(B, S, E), self.proj.weight, self.proj.bias)


class MLP(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        E = cfg.d_model
        self.fc = nn.Linear(E, cfg.mlp_ratio * E)
        self.proj = nn.Linear(cfg.mlp_ratio * E, E)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = T.bias_gelu(T.linear(x, self.fc.weight), self.fc.bias)
        return T.linear(h, self.proj.weight, self.proj.bias)


class Block(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.ln1 = FusedLayerNorm(cfg.d_model, cfg.ln_eps)
        self.attn = Attention(cfg)
        self.ln2 = FusedLayerNorm(cfg.d_model, cfg.ln_eps)
        self.mlp = MLP(cfg)
        self.dropout = cfg.dropout

    def forward(self, resid: torch.Tensor, delta: Optional[torch.Tensor], rope_cache=None):
        """Returns the new (residual stream, pending delta); the delta is added by the next
        fused LayerNorm."""
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


class GPT(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.cfg = cfg
        V, E = cfg.padded_vocab, cfg.d_model
        self.wte = nn.Embedding(V, E)
        self.wpe = nn.Embedding(cfg.max_seq_len, E) if cfg.pos_emb == "learned" else None
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = FusedLayerNorm(E, cfg.ln_eps)
        self.lm_head = None if cfg.tie_embeddings else nn.Linear(E, V, bias=False)
        self._rope = None
        if cfg.pos_emb == "rotary":
            rot = self.blocks[0].attn.rot
            cos, sin = T.rope_tables(cfg.max_seq_len, rot, cfg.rotary_base)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        std = self.cfg.init_std
        proj_std = std / math.sqrt(2 * self.cfg.n_layer)
        for name, p in self.named_parameters():
            if p.dim() < 2:
                if name.endswith("weight"):  # LayerNorm gains
                    nn.init.ones_(p)
                else:
                    nn.init.zeros_(p)
            elif name.endswith("proj.weight"):
                nn.init.normal_(p, 0.0, proj_std)
            else:
                nn.init.normal_(p, 0.0, std)

    def num_params(self, non_embedding: bool = True) -> int:
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.wte.weight.numel()
            if self.wpe is not None:
                n -= self.wpe.weight.numel()
        return n

    def flops_per_token(self, seq_len: Optional[int] = None) -> float:
        """Training FLOPs per token (fwd + bwd = 3x fwd), incl. causal attention (half of S^2)."""
        cfg = self.cfg
        S = seq_len or cfg.max_seq_len
        N = self.num_params(non_embedding=True)
        dense = 6 * N + 6 * cfg.d_model * cfg.padded_vocab
        attn = 6 * cfg.n_layer * cfg.d_model * S  # 12*L*E*S/2 for the causal half
        return float(dense + attn)

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
        w = self.wte.weight if self.lm_head is None else self.lm_head.weight
        logits = F.linear(h, w)
        if targets is None:
            return logits
        loss = T.cross_entropy(logits, targets, ignore_index=-100)
        return logits, loss


# ---------------------------------------------------------------------------------- pipeline form
def _init_like_gpt(module: nn.Module, cfg: GPTConfig) -> None:
    """GPT.reset_parameters' rules applied to one pipeline layer (same parameter names)."""
    std = cfg.init_std
    proj_std = std / math.sqrt(2 * cfg.n_layer)
    for name, p in module.named_parameters():
        if p.dim() < 2:
            nn.init.ones_(p) if name.endswith("weight") else nn.init.zeros_(p)
        elif name.endswith("proj.weight"):
            nn.init.normal_(p, 0.0, proj_std)
        else:
            nn.init.normal_(p, 0.0, std)


class EmbeddingPipe(nn.Module):
    """Token (+ learned position) embedding; tokens -> residual stream."""

    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Embedding(cfg.padded_vocab, cfg.d_model)
        self.wpe = nn.Embedding(cfg.max_seq_len, cfg.d_model) if cfg.pos_emb == "learned" else None
        _init_like_gpt(self, cfg)

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        x = self.wte(idx)
        if self.wpe is not None:
            x = x + self.wpe.weight[:idx.shape[1]].unsqueeze(0)
        return x


class BlockPipe(Block):
    """Transformer block on a pipeline activation: the residual stream, or (residual, pending
    delta) -- the delta is folded into the next fused LayerNorm, across stage boundaries too."""

    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__(cfg)
        self.rotary = cfg.pos_emb == "rotary"
        if self.rotary:
            cos, sin = T.rope_tables(cfg.max_seq_len, self.attn.rot, cfg.rotary_base)
            self.register_buffer("rope_cos", cos, persistent=False)
            self.register_buffer("rope_sin", sin, persistent=False)
        _init_like_gpt(self, cfg)

    def forward(self, x):  # type: ignore[override]
        resid, delta = (x, None) if isinstance(x, torch.Tensor) else x
        rope = (self.rope_cos, self.rope_sin) if self.rotary else None
        return super().forward(resid, delta, rope)


class FinalNormPipe(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.ln_f = FusedLayerNorm(cfg.d_model, cfg.ln_eps)

    def forward(self, x) -> torch.Tensor:
        if isinstance(x, torch.Tensor):
            return self.ln_f(x)
        h, _ = self.ln_f(x[0], residual=x[1])
        return h


class LMHeadPipe(nn.Module):
    def __init__(self, cfg: GPTConfig) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cfg.padded_vocab, cfg.d_model))
        nn.init.normal_(self.weight, 0.0, cfg.init_std)

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        return F.linear(h, self.weight)


def _tied_head(module: nn.Module, h: torch.Tensor) -> torch.Tensor:
    return F.linear(h, module.wte.weight)


def pipeline_loss(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    return T.cross_entropy(logits, targets, ignore_index=-100)


def pipeline_specs(cfg: GPTConfig) -> list:
    """GPT as a layer list for :class:`~determined_clone_amd.parallel.pipeline.PipelineModule`
    (the GPT-NeoX pipe form the reference's gpt_neox example trains with pipe_parallel_size=2):
    embedding, blocks, final LayerNorm, LM head (tied to the embedding table when
    ``cfg.tie_embeddings``: a TiedLayerSpec whose gradient is summed across the first and last
    stage)."""
    from determined_clone_amd.parallel.pipeline import LayerSpec, TiedLayerSpec

    if cfg.tie_embeddings:
        embed = TiedLayerSpec("embed", EmbeddingPipe, cfg, tied_weight_attr="wte.weight")
        head = TiedLayerSpec("embed", EmbeddingPipe, cfg, forward_fn=_tied_head,
                             tied_weight_attr="wte.weight")
    else:
        embed, head = LayerSpec(EmbeddingPipe, cfg), LayerSpec(LMHeadPipe, cfg)
    return [embed] + [LayerSpec(BlockPipe, cfg) for _ in range(cfg.n_layer)] + \
        [LayerSpec(FinalNormPipe, cfg), head]


def cast_for_mi355x(model: nn.Module, dtype: torch.dtype = torch.bfloat16) -> nn.Module:
    """GEMM / embedding weights -> ``dtype``; modules marked ``keep_fp32`` (LayerNorm, BatchNorm)
    keep fp32 parameters (the fused kernels read them as fp32)."""
    for m in model.modules():
        keep = getattr(m, "keep_fp32", False) or isinstance(m, (nn.LayerNorm, nn.GroupNorm,
                                                                 nn.modules.batchnorm._BatchNorm))
        for name, p in list(m.named_parameters(recurse=False)):
            if p.is_floating_point() and not keep:
                p.data = p.data.to(dtype)
    return model


def gpt2(name: str = "gpt2-medium", **overrides) -> GPT:
    return GPT(config_for(name, **overrides))
