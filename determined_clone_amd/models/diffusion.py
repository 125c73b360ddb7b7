"""Latent diffusion (Stable-Diffusion-style) model family, written for MI355X.

Reference: `examples/diffusion/textual_inversion_stable_diffusion` (``detsd/``), which drives
HF ``diffusers`` (UNet2DConditionModel, AutoencoderKL, DDPM/PNDM/DDIM schedulers,
StableDiffusionPipeline) and a CLIP text encoder. ``diffusers`` and pretrained weights are not in
this image, so the architecture is defined here from the published design (latent diffusion:
VAE with 8x spatial compression, a text-conditioned UNet with cross-attention, classifier-free
guidance) and runs with random-init weights:

* every attention (UNet self/cross attention, VAE mid-block attention, the causal text encoder)
  uses 64-wide heads, so on the GPU it runs on the hand-written MFMA flash-attention kernels of
  ``ops/csrc/attention.hip`` (bf16, never materialising the score matrix; ``Sq != Sk`` for the
  77-token cross attention) -- the SD-2 convention (``attention_head_dim=64``) rather than SD-1's
  8 fixed heads, which would give 40/80/160-wide heads;
* activations are NHWC bf16 on the GPU (MIOpen NHWC implicit-GEMM convolutions); every
  GroupNorm (+ SiLU) is one fused NHWC HIP kernel family (``ops/csrc/groupnorm.hip``), statistics in
  fp32/fp64;
* ``UNetConfig.sd()`` is the SD-2-base UNet shape (320/640/1280/1280 channels, 2 layers per block,
  1024-wide context), ``.tiny()`` a small one for tests.

Also here: the noise schedulers (DDPM training noise, DDIM and PNDM/PLMS sampling), a
deterministic hashing word tokenizer standing in for CLIP's BPE vocabulary (not available
offline), :class:`ExtendedEmbedding` (frozen vocabulary + trainable concept rows, as the
reference's ``detsd/layers.py``) and :class:`LatentDiffusionPipeline` (text -> image with
classifier-free guidance).
"""
import math
import re
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import conv as conv_ops
from determined_clone_amd.ops import transformer as tops
from determined_clone_amd.ops.groupnorm import GroupNormAct
from determined_clone_amd.ops.transformer import flash_attention, reference_attention


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    """[B, S, H, 64] attention: MFMA flash-attention kernels on the GPU (bf16), fp32 oracle on
    CPU."""
    if q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128):
        return flash_attention(q.contiguous(), k.contiguous(), v.contiguous(), causal=causal)
    return reference_attention(q.float(), k.float(), v.float(), causal).to(q.dtype)


class Conv2d(nn.Conv2d):
    """Convolution whose weight/bias gradients run on the side HIP stream (``ops/conv.py``)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return conv_ops.spatial_conv(self, x)


class Linear(nn.Linear):
    """Linear layer with gradient accumulation into flat ``.grad`` views and side-stream weight
    gradients on the GPU (``ops/transformer.py``)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return tops.linear(x, self.weight, self.bias)


class LayerNorm(nn.LayerNorm):
    """LayerNorm on the fused HIP kernel (fp32 statistics) on the GPU."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return tops.layer_norm(x, self.weight, self.bias, self.eps)
        return super().forward(x)


def _groups(ch: int, want: int) -> int:
    g = min(want, ch)
    while ch % g:
        g -= 1
    return g


# ============================================================================ configs
@dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: Tuple[int, ...] = (320, 640, 1280, 1280)
    cross_attn: Tuple[bool, ...] = (True, True, True, False)
    layers_per_block: int = 2
    cross_attention_dim: int = 1024
    head_dim: int = 64
    norm_groups: int = 32

    @classmethod
    def sd(cls) -> "UNetConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "UNetConfig":
        return cls(block_out_channels=(64, 128), cross_attn=(True, False), layers_per_block=1,
                   cross_attention_dim=64, head_dim=64, norm_groups=32)


@dataclass
class VAEConfig:
    in_channels: int = 3
    latent_channels: int = 4
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_groups: int = 32
    scaling_factor: float = 0.18215

    @classmethod
    def sd(cls) -> "VAEConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "VAEConfig":
        return cls(block_out_channels=(32, 64, 64, 64), layers_per_block=1)


@dataclass
class TextConfig:
    vocab_size: int = 49408
    max_length: int = 77
    width: int = 1024
    layers: int = 23
    head_dim: int = 64

    @classmethod
    def sd(cls) -> "TextConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "TextConfig":
        return cls(vocab_size=1000, max_length=16, width=64, layers=2)


@dataclass
class LDMConfig:
    unet: UNetConfig = field(default_factory=UNetConfig)
    vae: VAEConfig = field(default_factory=VAEConfig)
    text: TextConfig = field(default_factory=TextConfig)

    @classmethod
    def preset(cls, name: str) -> "LDMConfig":
        if name in ("sd", "sd2-base"):
            return cls(UNetConfig.sd(), VAEConfig.sd(), TextConfig.sd())
        if name == "tiny":
            return cls(UNetConfig.tiny(), VAEConfig.tiny(), TextConfig.tiny())
        raise ValueError(f"unknown latent-diffusion preset {name!r} (sd2-base | tiny)")


# ============================================================================ building blocks
def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000.0) -> torch.Tensor:
    """Sinusoidal timestep features, cos first (the diffusers ``flip_sin_to_cos=True`` layout)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(half, device=t.device, dtype=torch.float32) / half)
    args = t.float()[:, None] * freqs[None]
    return torch.cat([torch.cos(args), torch.sin(args)], dim=-1)


class ResnetBlock(nn.Module):
    def __init__(self, cin: int, cout: int, temb: Optional[int], groups: int) -> None:
        super().__init__()
        self.norm1 = GroupNormAct(_groups(cin, groups), cin, eps=1e-5 if temb else 1e-6, act=True)
        self.conv1 = Conv2d(cin, cout, 3, padding=1)
        self.time_emb_proj = Linear(temb, cout) if temb else None
        self.norm2 = GroupNormAct(_groups(cout, groups), cout, eps=1e-5 if temb else 1e-6, act=True)
        self.conv2 = Conv2d(cout, cout, 3, padding=1)
        self.shortcut = Conv2d(cin, cout, 1) if cin != cout else None

    def forward(self, x: torch.Tensor, temb: Optional[torch.Tensor] = None) -> torch.Tensor:
        h = self.conv1(self.norm1(x))  # GroupNorm + SiLU: one fused NHWC kernel on the GPU
        if self.time_emb_proj is not None and temb is not None:
            h = h + self.time_emb_proj(F.silu(temb)).to(h.dtype)[:, :, None, None]
        h = self.conv2(self.norm2(h))
        return (x if self.shortcut is None else self.shortcut(x)) + h


class MultiHeadAttention(nn.Module):
    """Self- (``ctx_dim=None``) or cross-attention over [B, S, C] tokens, 64-wide heads."""

    def __init__(self, dim: int, head_dim: int, ctx_dim: Optional[int] = None, bias: bool = False,
                 causal: bool = False) -> None:
        super().__init__()
        self.heads, self.head_dim, self.causal = max(1, dim // head_dim), head_dim, causal
        inner = self.heads * head_dim
        self.to_q = Linear(dim, inner, bias=bias)
        self.to_k = Linear(ctx_dim or dim, inner, bias=bias)
        self.to_v = Linear(ctx_dim or dim, inner, bias=bias)
        self.to_out = Linear(inner, dim)

    def forward(self, x: torch.Tensor, ctx: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = x if ctx is None else ctx
        B, S, _ = x.shape
        q = self.to_q(x).view(B, S, self.heads, self.head_dim)
        k = self.to_k(c).view(B, c.shape[1], self.heads, self.head_dim)
        v = self.to_v(c).view(B, c.shape[1], self.heads, self.head_dim)
        o = attention(q, k, v, self.causal)
        return self.to_out(o.reshape(B, S, -1))


class GEGLU(nn.Module):
    def __init__(self, dim: int, mult: int = 4) -> None:
        super().__init__()
        self.proj = Linear(dim, dim * mult * 2)
        self.out = Linear(dim * mult, dim)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h, gate = self.proj(x).chunk(2, dim=-1)
        return self.out(h * F.gelu(gate))


class TransformerBlock(nn.Module):
    def __init__(self, dim: int, head_dim: int, ctx_dim: int) -> None:
        super().__init__()
        self.norm1, self.attn1 = LayerNorm(dim), MultiHeadAttention(dim, head_dim)
        self.norm2, self.attn2 = LayerNorm(dim), MultiHeadAttention(dim, head_dim, ctx_dim)
        self.norm3, self.ff = LayerNorm(dim), GEGLU(dim)

    def forward(self, x: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        x = x + self.attn1(self.norm1(x))
        x = x + self.attn2(self.norm2(x), ctx)
        return x + self.ff(self.norm3(x))


class SpatialTransformer(nn.Module):
    """GroupNorm -> tokens -> transformer block (self + cross attention + GEGLU) -> residual."""

    def __init__(self, ch: int, head_dim: int, ctx_dim: int, groups: int) -> None:
        super().__init__()
        self.norm = GroupNormAct(_groups(ch, groups), ch, eps=1e-6)
        self.proj_in = Linear(ch, ch)
        self.block = TransformerBlock(ch, head_dim, ctx_dim)
        self.proj_out = Linear(ch, ch)

    def forward(self, x: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x.shape
        h = self.norm(x).permute(0, 2, 3, 1).reshape(B, H * W, C)  # NHWC: a view, no copy
        h = self.proj_out(self.block(self.proj_in(h), ctx))
        return x + h.view(B, H, W, C).permute(0, 3, 1, 2)


class Downsample(nn.Module):
    def __init__(self, ch: int, asym_pad: bool = False) -> None:
        super().__init__()
        self.asym = asym_pad
        self.conv = Conv2d(ch, ch, 3, stride=2, padding=0 if asym_pad else 1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.asym:
            x = F.pad(x, (0, 1, 0, 1))
        return self.conv(x)


class Upsample(nn.Module):
    def __init__(self, ch: int) -> None:
        super().__init__()
        self.conv = Conv2d(ch, ch, 3, padding=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


# ============================================================================ UNet
class UNet2DCondition(nn.Module):
    def __init__(self, cfg: UNetConfig) -> None:
        super().__init__()
        self.cfg = cfg
        ch = cfg.block_out_channels
        temb = ch[0] * 4
        g, hd, cd = cfg.norm_groups, cfg.head_dim, cfg.cross_attention_dim
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_mlp = nn.Sequential(Linear(ch[0], temb), nn.SiLU(), Linear(temb, temb))
        self.down = nn.ModuleList()
        skips = [ch[0]]
        cin = ch[0]
        for i, c in enumerate(ch):
            blk = nn.Module()
            blk.resnets = nn.ModuleList()
            blk.attns = nn.ModuleList()
            for _ in range(cfg.layers_per_block):
                blk.resnets.append(ResnetBlock(cin, c, temb, g))
                blk.attns.append(SpatialTransformer(c, hd, cd, g) if cfg.cross_attn[i] else nn.Identity())
                cin = c
                skips.append(c)
            blk.downsample = Downsample(c) if i < len(ch) - 1 else None
            if blk.downsample is not None:
                skips.append(c)
            self.down.append(blk)
        self.mid_res1 = ResnetBlock(ch[-1], ch[-1], temb, g)
        self.mid_attn = SpatialTransformer(ch[-1], hd, cd, g)
        self.mid_res2 = ResnetBlock(ch[-1], ch[-1], temb, g)
        self.up = nn.ModuleList()
        rev = list(reversed(ch))
        cross_rev = list(reversed(cfg.cross_attn))
        cin = ch[-1]
        for i, c in enumerate(rev):
            blk = nn.Module()
            blk.resnets = nn.ModuleList()
            blk.attns = nn.ModuleList()
            for _ in range(cfg.layers_per_block + 1):
                blk.resnets.append(ResnetBlock(cin + skips.pop(), c, temb, g))
                blk.attns.append(SpatialTransformer(c, hd, cd, g) if cross_rev[i] else nn.Identity())
                cin = c
            blk.upsample = Upsample(c) if i < len(rev) - 1 else None
            self.up.append(blk)
        self.norm_out = GroupNormAct(_groups(ch[0], g), ch[0], eps=1e-5, act=True)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        if t.dim() == 0:
            t = t.expand(x.shape[0])
        emb = self.time_mlp(timestep_embedding(t, self.cfg.block_out_channels[0]).to(self.conv_in.weight.dtype))
        ctx = ctx.to(self.conv_in.weight.dtype)
        h = self.conv_in(x)
        skips = [h]
        for blk in self.down:
            for res, attn in zip(blk.resnets, blk.attns):
                h = res(h, emb)
                h = h if isinstance(attn, nn.Identity) else attn(h, ctx)
                skips.append(h)
            if blk.downsample is not None:
                h = blk.downsample(h)
                skips.append(h)
        h = self.mid_res2(self.mid_attn(self.mid_res1(h, emb), ctx), emb)
        for blk in self.up:
            for res, attn in zip(blk.resnets, blk.attns):
                h = res(torch.cat([h, skips.pop()], dim=1), emb)
                h = h if isinstance(attn, nn.Identity) else attn(h, ctx)
            if blk.upsample is not None:
                h = blk.upsample(h)
        return self.conv_out(self.norm_out(h))


# ============================================================================ VAE
class _VAEAttention(nn.Module):
    def __init__(self, ch: int, groups: int) -> None:
        super().__init__()
        self.norm = GroupNormAct(_groups(ch, groups), ch, eps=1e-6)
        self.attn = MultiHeadAttention(ch, 64, bias=True)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x.shape
        h = self.norm(x).permute(0, 2, 3, 1).reshape(B, H * W, C)
        return x + self.attn(h).view(B, H, W, C).permute(0, 3, 1, 2)


class AutoencoderKL(nn.Module):
    """KL-regularised autoencoder: 8x spatial compression to ``latent_channels`` (SD's VAE shape)."""

    def __init__(self, cfg: VAEConfig) -> None:
        super().__init__()
        self.cfg = cfg
        ch, g, n = cfg.block_out_channels, cfg.norm_groups, cfg.layers_per_block
        self.enc_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.enc_blocks = nn.ModuleList()
        cin = ch[0]
        for i, c in enumerate(ch):
            mods = [ResnetBlock(cin if j == 0 else c, c, None, g) for j in range(n)]
            if i < len(ch) - 1:
                mods.append(Downsample(c, asym_pad=True))
            self.enc_blocks.append(nn.ModuleList(mods))
            cin = c
        self.enc_mid = nn.ModuleList([ResnetBlock(ch[-1], ch[-1], None, g), _VAEAttention(ch[-1], g),
                                      ResnetBlock(ch[-1], ch[-1], None, g)])
        self.enc_norm = GroupNormAct(_groups(ch[-1], g), ch[-1], eps=1e-6, act=True)
        self.enc_out = Conv2d(ch[-1], 2 * cfg.latent_channels, 3, padding=1)
        self.quant_conv = Conv2d(2 * cfg.latent_channels, 2 * cfg.latent_channels, 1)
        self.post_quant_conv = Conv2d(cfg.latent_channels, cfg.latent_channels, 1)
        self.dec_in = Conv2d(cfg.latent_channels, ch[-1], 3, padding=1)
        self.dec_mid = nn.ModuleList([ResnetBlock(ch[-1], ch[-1], None, g), _VAEAttention(ch[-1], g),
                                      ResnetBlock(ch[-1], ch[-1], None, g)])
        self.dec_blocks = nn.ModuleList()
        rev = list(reversed(ch))
        cin = ch[-1]
        for i, c in enumerate(rev):
            mods = [ResnetBlock(cin if j == 0 else c, c, None, g) for j in range(n + 1)]
            if i < len(rev) - 1:
                mods.append(Upsample(c))
            self.dec_blocks.append(nn.ModuleList(mods))
            cin = c
        self.dec_norm = GroupNormAct(_groups(ch[0], g), ch[0], eps=1e-6, act=True)
        self.dec_out = Conv2d(ch[0], cfg.in_channels, 3, padding=1)

    def encode(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Images in [-1, 1] -> (mean, logvar) of the latent posterior."""
        h = self.enc_in(x)
        for blk in self.enc_blocks:
            for m in blk:
                h = m(h)
        for m in self.enc_mid:
            h = m(h)
        moments = self.quant_conv(self.enc_out(self.enc_norm(h)))
        mean, logvar = moments.chunk(2, dim=1)
        return mean, logvar.clamp(-30.0, 20.0)

    def sample_latents(self, x: torch.Tensor, generator: Optional[torch.Generator] = None) -> torch.Tensor:
        mean, logvar = self.encode(x)
        eps = torch.randn(mean.shape, generator=generator, device=mean.device, dtype=mean.dtype)
        return (mean + torch.exp(0.5 * logvar) * eps) * self.cfg.scaling_factor

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        h = self.dec_in(self.post_quant_conv(z / self.cfg.scaling_factor))
        for m in self.dec_mid:
            h = m(h)
        for blk in self.dec_blocks:
            for m in blk:
                h = m(h)
        return self.dec_out(self.dec_norm(h))


# ============================================================================ text encoder
class ExtendedEmbedding(nn.Module):
    """Frozen vocabulary rows + a separate, trainable table for ids >= ``vocab_size`` (the new
    concept tokens of textual inversion)."""

    def __init__(self, original: nn.Embedding, new_weights: torch.Tensor) -> None:
        super().__init__()
        self.original = original
        self.vocab = original.num_embeddings
        self.new_embedding = nn.Embedding(new_weights.shape[0], new_weights.shape[1])
        with torch.no_grad():
            self.new_embedding.weight.copy_(new_weights)

    @property
    def weight(self) -> torch.Tensor:
        return torch.cat([self.original.weight, self.new_embedding.weight], dim=0)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        is_new = ids >= self.vocab
        out = self.original(ids.clamp(max=self.vocab - 1))
        if bool(is_new.any()):
            new = self.new_embedding((ids - self.vocab).clamp(min=0)).to(out.dtype)
            out = torch.where(is_new[..., None], new, out)
        return out


class TextEncoder(nn.Module):
    """CLIP-style causal text transformer (pre-LN, quick-GELU MLP), last hidden state out."""

    def __init__(self, cfg: TextConfig) -> None:
        super().__init__()
        self.cfg = cfg
        d = cfg.width
        self.token_embedding: nn.Module = nn.Embedding(cfg.vocab_size, d)
        self.position_embedding = nn.Embedding(cfg.max_length, d)
        self.layers = nn.ModuleList()
        for _ in range(cfg.layers):
            layer = nn.Module()
            layer.ln1 = LayerNorm(d)
            layer.attn = MultiHeadAttention(d, cfg.head_dim, bias=True, causal=True)
            layer.ln2 = LayerNorm(d)
            layer.fc1 = Linear(d, 4 * d)
            layer.fc2 = Linear(4 * d, d)
            self.layers.append(layer)
        self.final_ln = LayerNorm(d)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        pos = torch.arange(ids.shape[1], device=ids.device)
        h = self.token_embedding(ids) + self.position_embedding(pos)[None].to(self.final_ln.weight.dtype)
        for layer in self.layers:
            h = h + layer.attn(layer.ln1(h))
            f = layer.fc1(layer.ln2(h))
            h = h + layer.fc2(f * torch.sigmoid(1.702 * f))
        return self.final_ln(h)

    def add_concept_rows(self, init_rows: torch.Tensor) -> None:
        """Append trainable rows (initialised from ``init_rows``) after the vocabulary."""
        base = self.token_embedding.original if isinstance(self.token_embedding, ExtendedEmbedding) \
            else self.token_embedding
        prev = self.token_embedding.new_embedding.weight.data if isinstance(
            self.token_embedding, ExtendedEmbedding) else init_rows[:0]
        self.token_embedding = ExtendedEmbedding(base, torch.cat([prev, init_rows.to(prev.device)], 0))


class HashTokenizer:
    """Word-level tokenizer with a fixed hashed vocabulary (CLIP's BPE merges/vocab files are not
    available offline). ``[BOS] words... [EOS] [PAD]...`` to ``max_length``; added tokens get ids
    after the base vocabulary, like ``tokenizer.add_tokens``."""

    def __init__(self, vocab_size: int, max_length: int) -> None:
        self.vocab_size = vocab_size
        self.model_max_length = max_length
        self.bos, self.eos = vocab_size - 2, vocab_size - 1
        self.pad = self.eos
        self.added: Dict[str, int] = {}

    def __len__(self) -> int:
        return self.vocab_size + len(self.added)

    def add_tokens(self, tokens: Sequence[str]) -> List[int]:
        ids = []
        for t in tokens:
            if t not in self.added:
                self.added[t] = self.vocab_size + len(self.added)
            ids.append(self.added[t])
        return ids

    def word_ids(self, text: str) -> List[int]:
        out: List[int] = []
        pieces = re.findall(r"<[^>]+>|[\w'-]+|[^\w\s]", text.lower())
        for w in pieces:
            if w in self.added:
                out.append(self.added[w])
            else:
                out.append(zlib.crc32(w.encode()) % (self.vocab_size - 2))
        return out

    def __call__(self, texts: Sequence[str]) -> torch.Tensor:
        rows = []
        for t in texts:
            ids = [self.bos] + self.word_ids(t)[: self.model_max_length - 2] + [self.eos]
            rows.append(ids + [self.pad] * (self.model_max_length - len(ids)))
        return torch.tensor(rows, dtype=torch.long)


# ============================================================================ schedulers
def make_betas(n: int, beta_start: float, beta_end: float, schedule: str) -> torch.Tensor:
    if schedule == "scaled_linear":
        return torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n, dtype=torch.float64) ** 2
    if schedule == "linear":
        return torch.linspace(beta_start, beta_end, n, dtype=torch.float64)
    raise ValueError(f"unknown beta_schedule {schedule!r}")


class DDPMScheduler:
    """Forward (noising) process used for training."""

    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.00085,
                 beta_end: float = 0.012, beta_schedule: str = "scaled_linear") -> None:
        self.num_train_timesteps = num_train_timesteps
        self.betas = make_betas(num_train_timesteps, beta_start, beta_end, beta_schedule)
        self.alphas_cumprod = torch.cumprod(1.0 - self.betas, 0)

    def add_noise(self, x0: torch.Tensor, noise: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        ac = self.alphas_cumprod.to(x0.device)[t].float()
        shape = (-1,) + (1,) * (x0.dim() - 1)
        return ac.sqrt().view(shape).to(x0.dtype) * x0 + (1 - ac).sqrt().view(shape).to(x0.dtype) * noise


class DDIMScheduler(DDPMScheduler):
    """Deterministic DDIM sampling (eta = 0)."""

    def set_timesteps(self, n: int) -> List[int]:
        self.num_inference_steps = n
        ratio = self.num_train_timesteps // n
        self.timesteps = [i * ratio + 1 for i in reversed(range(n))]
        return self.timesteps

    def step(self, eps: torch.Tensor, t: int, x: torch.Tensor) -> torch.Tensor:
        prev = t - self.num_train_timesteps // self.num_inference_steps
        a_t = float(self.alphas_cumprod[t])
        a_p = float(self.alphas_cumprod[prev]) if prev >= 0 else float(self.alphas_cumprod[0])
        x0 = (x - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
        return math.sqrt(a_p) * x0 + math.sqrt(1 - a_p) * eps


class PNDMScheduler(DDPMScheduler):
    """Pseudo-numerical (PLMS, linear multistep) sampling of Liu et al. 2022, the Stable Diffusion
    default (``skip_prk_steps``): the first step is a 2nd-order corrector, then 2/3/4-step
    Adams-Bashforth combinations of past noise predictions."""

    def set_timesteps(self, n: int) -> List[int]:
        self.num_inference_steps = n
        self.ratio = self.num_train_timesteps // n
        base = [i * self.ratio + 1 for i in range(n)]
        plms = base[:-1] + base[-2:-1] + base[-1:]
        self.timesteps = list(reversed(plms))
        self.ets: List[torch.Tensor] = []
        self.counter = 0
        self.cur_sample: Optional[torch.Tensor] = None
        return self.timesteps

    def _prev(self, x: torch.Tensor, t: int, prev: int, eps: torch.Tensor) -> torch.Tensor:
        a_t = float(self.alphas_cumprod[t])
        a_p = float(self.alphas_cumprod[prev]) if prev >= 0 else float(self.alphas_cumprod[0])
        b_t, b_p = 1 - a_t, 1 - a_p
        coeff = math.sqrt(a_p / a_t)
        denom = a_t * math.sqrt(b_p) + math.sqrt(a_t * b_t * a_p)
        return coeff * x - (a_p - a_t) * eps / denom

    def step(self, eps: torch.Tensor, t: int, x: torch.Tensor) -> torch.Tensor:
        prev = t - self.ratio
        if self.counter != 1:
            self.ets = self.ets[-3:] + [eps]
        else:
            prev, t = t, t + self.ratio
        e = self.ets
        if len(e) == 1 and self.counter == 0:
            out, self.cur_sample = e[-1], x
        elif len(e) == 1 and self.counter == 1:
            out, x, self.cur_sample = (eps + e[-1]) / 2, self.cur_sample, None
        elif len(e) == 2:
            out = (3 * e[-1] - e[-2]) / 2
        elif len(e) == 3:
            out = (23 * e[-1] - 16 * e[-2] + 5 * e[-3]) / 12
        else:
            out = (55 * e[-1] - 59 * e[-2] + 37 * e[-3] - 9 * e[-4]) / 24
        self.counter += 1
        return self._prev(x, t, prev, out)


SCHEDULERS = {"ddim": DDIMScheduler, "pndm": PNDMScheduler}


# ============================================================================ model + pipeline
def to_mi355x_layout(module: nn.Module, device: torch.device, dtype: torch.dtype = torch.bfloat16):
    """bf16 weights + NHWC on the GPU, GroupNorm affine parameters kept fp32 (read as fp32 by the
    fused NHWC GroupNorm kernels)."""
    module.to(device=device, dtype=dtype)
    if device.type == "cuda":
        module.to(memory_format=torch.channels_last)
        for m in module.modules():
            if isinstance(m, GroupNormAct):
                m.float()
    return module


class LatentDiffusion(nn.Module):
    def __init__(self, cfg: LDMConfig) -> None:
        super().__init__()
        self.cfg = cfg
        self.unet = UNet2DCondition(cfg.unet)
        self.vae = AutoencoderKL(cfg.vae)
        self.text_encoder = TextEncoder(cfg.text)
        self.tokenizer = HashTokenizer(cfg.text.vocab_size, cfg.text.max_length)

    def to_mi355x_layout(self, device: torch.device, dtype: torch.dtype = torch.bfloat16) -> "LatentDiffusion":
        """GPU layout: bf16 weights, NHWC convolutions; GroupNorm affine parameters stay fp32 (the
        fused NHWC GroupNorm kernels read them as fp32)."""
        return to_mi355x_layout(self, device, dtype)

    def encode_text(self, texts: Sequence[str]) -> torch.Tensor:
        ids = self.tokenizer(texts).to(self.text_encoder.final_ln.weight.device)
        return self.text_encoder(ids)


class LatentDiffusionPipeline:
    """Text -> image: classifier-free guidance over the UNet's noise prediction, scheduler steps in
    latent space, VAE decode (reference: diffusers ``StableDiffusionPipeline`` as used by
    ``detsd/pipeline.py``)."""

    def __init__(self, model: LatentDiffusion, scheduler: str = "pndm", beta_start: float = 0.00085,
                 beta_end: float = 0.012, beta_schedule: str = "scaled_linear") -> None:
        self.model = model
        self.scheduler = SCHEDULERS[scheduler](1000, beta_start, beta_end, beta_schedule)

    @torch.no_grad()
    def __call__(self, prompts: Sequence[str], num_inference_steps: int = 50,
                 guidance_scale: float = 7.5, height: int = 512, width: int = 512,
                 generator: Optional[torch.Generator] = None) -> torch.Tensor:
        m = self.model
        dev = m.text_encoder.final_ln.weight.device
        dtype = m.unet.conv_in.weight.dtype
        cond = m.encode_text(list(prompts))
        uncond = m.encode_text([""] * len(prompts))
        ctx = torch.cat([uncond, cond])
        f = 2 ** (len(m.cfg.vae.block_out_channels) - 1)
        lat = torch.randn((len(prompts), m.cfg.unet.in_channels, height // f, width // f),
                          generator=generator, device="cpu" if generator is None else generator.device)
        lat = lat.to(dev, torch.float32)
        if dev.type == "cuda":
            lat = lat.contiguous(memory_format=torch.channels_last)
        for t in self.scheduler.set_timesteps(num_inference_steps):
            x_in = torch.cat([lat, lat]).to(dtype)
            eps = m.unet(x_in, torch.full((x_in.shape[0],), t, device=dev), ctx).float()
            e_u, e_c = eps.chunk(2)
            lat = self.scheduler.step(e_u + guidance_scale * (e_c - e_u), t, lat)
        img = m.vae.decode(lat.to(dtype)).float()
        return ((img.clamp(-1, 1) + 1) * 127.5).round().to(torch.uint8).permute(0, 2, 3, 1).cpu()
