"""Transformer hot ops: fused residual-add + LayerNorm, bias + GELU, rotary embedding, flash
attention.

GPU path: `ops/csrc/transformer.hip` and `ops/csrc/attention.hip` (MFMA 16x16x32 bf16). CPU path
(and fp32 oracle for the GPU numerics tests): plain PyTorch.

These replace the fused kernels the reference's GPT-NeoX DeepSpeedTrial example gets from
DeepSpeed / apex (reference: examples/deepspeed/gpt_neox/gpt2_trial.py, which builds the
NeoX model with `fused_softmax`, `scaled_upper_triang_masked_softmax` and apex FusedLayerNorm).
Layouts are the ones the model produces without copies: activations [..., D] row-major,
attention operands [B, S, H, Dh] (slices of the fused QKV projection are accepted as-is).
"""
import contextlib
import math
import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from determined_clone_amd.ops import _ext, _grad

# ----------------------------------------------------------------------------- references


def reference_layer_norm(x, weight, bias, eps=1e-5, residual=None):
    s = x if residual is None else x + residual
    y = F.layer_norm(s.float(), (s.shape[-1],), None if weight is None else weight.float(),
                     None if bias is None else bias.float(), eps).to(x.dtype)
    return y if residual is None else (y, s)


def reference_bias_gelu(x, bias):
    h = x.float() if bias is None else x.float() + bias.float()
    return F.gelu(h, approximate="tanh").to(x.dtype)


def rope_tables(seq_len: int, rot_dim: int, base: float = 10000.0, device=None):
    """cos/sin tables [S, rot_dim/2] (fp32) for the rotate-half convention."""
    inv = 1.0 / (base ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    fr = torch.outer(t, inv)
    return fr.cos().float().to(device), fr.sin().float().to(device)


def reference_rope(x, cos, sin, rot_dim: Optional[int] = None):
    """x: [B, S, H, D]."""
    D = x.shape[-1]
    rot = rot_dim or D
    half = rot // 2
    xf = x.float()
    c = cos[: x.shape[1], :half].to(x.device)[None, :, None, :]
    s = sin[: x.shape[1], :half].to(x.device)[None, :, None, :]
    a, b, rest = xf[..., :half], xf[..., half:rot], xf[..., rot:]
    out = torch.cat([a * c - b * s, b * c + a * s, rest], dim=-1)
    return out.to(x.dtype)


def reference_attention(q, k, v, causal=True, scale=None, key_lengths=None):
    """q [B, S, H, D], k/v [B, Sk, Hkv, D] with Hkv dividing H (grouped-query attention: query
    head h reads K/V head h // (H / Hkv)) -> [B, S, H, D] (fp32 math). ``key_lengths`` [B]: keys
    at or past it are masked (right padding), clamped to at least one key like the kernels."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if k.shape[2] != q.shape[2]:
        g = q.shape[2] // k.shape[2]
        k, v = k.repeat_interleave(g, dim=2), v.repeat_interleave(g, dim=2)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        S = s.shape[-1]
        mask = torch.ones(s.shape[-2], S, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    if key_lengths is not None:
        kl = key_lengths.to(s.device).long().clamp_min(1)
        pad = torch.arange(s.shape[-1], device=s.device)[None, :] >= kl[:, None]
        s = s.masked_fill(pad[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.matmul(p, vf).transpose(1, 2).to(q.dtype)


# ----------------------------------------------------------------------------- autograd


def _gpu_ok(x: torch.Tensor, div: int = 8) -> bool:
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and x.shape[-1] % div == 0


def _f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if t is None:
        return None
    return t if t.dtype == torch.float32 and t.is_contiguous() else t.float().contiguous()


# DCA_FUSE_LN_BIAS_GRAD=1: the out-projection bias gradients come out of the LayerNorm backward
# (its dx column sums, +0.6 us per call in isolation) instead of a separate column reduction. OFF by
# default: the GPT-2-medium step measured 0.6 % slower with it (381.6k vs 383.9k tok/s, same box,
# profiles/round5_ln_bwd_bias_grad_fusion_ab.txt) -- on the main stream the separate memory-bound
# reduction pairs better with the side stream's weight-gradient GEMMs than the next dX GEMM does.
FUSE_LN_BIAS_GRAD = os.environ.get("DCA_FUSE_LN_BIAS_GRAD", "0") == "1"
LN_BIAS_GRAD_HITS = [0]


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps):
        C = _ext.load()
        x = x.contiguous()
        res = residual.contiguous() if residual is not None else None
        if res is not None and res.dtype != x.dtype:
            res = res.to(x.dtype)
        y, s, mean, rstd = C.ln_fwd(x, res, _f32(weight), _f32(bias), eps, res is not None)
        # Backward needs the normalised input: the residual sum when fused, else x.
        ctx.save_for_backward(s if res is not None else x, weight, mean, rstd)
        ctx.has_res = res is not None
        ctx.w_dtype = weight.dtype if weight is not None else None
        ctx.params = (weight, bias)
        # pre-LN block: the residual input is the output of a ``linear`` (attention / MLP out
        # projection) whose dy is exactly this LayerNorm's dx -- its bias gradient is reduced in
        # the LN backward pass instead of by a separate column sum (``_Linear.backward``)
        ctx.bias_node = residual.grad_fn if (FUSE_LN_BIAS_GRAD and res is not None and res is residual and
                                             type(residual.grad_fn).__name__ == "_LinearBackward") else None
        if res is not None:
            return y, s
        return y

    @staticmethod
    def backward(ctx, dy, dsum=None):
        xin, weight, mean, rstd = ctx.saved_tensors
        need_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        acc_g, acc_b = (_grad.target(ctx.params[0]), _grad.target(ctx.params[1])) if need_w else (None, None)
        if acc_g is None or acc_b is None or acc_g.dtype != acc_b.dtype:
            acc_g = acc_b = None
        node, acc_cs = ctx.bias_node, None
        ctx.bias_node = None
        if node is not None and ctx.needs_input_grad[1] and node.needs_input_grad[2] and \
                node.params[1] is not None:
            acc_cs = _grad.target(node.params[1])
        dx, dg, db = _ext.load().ln_bwd(dy, xin, _f32(weight), mean, rstd,
                                        dsum if ctx.has_res else None, need_w, acc_g, acc_b, acc_cs)
        if acc_cs is not None:
            node._dca_bias_given = dx  # (+)= dx.sum(rows) is already in the bias .grad
            LN_BIAS_GRAD_HITS[0] += 1
        if acc_g is not None:
            need_w = False  # accumulated into .grad in-kernel
        if need_w:
            dg = dg.to(ctx.w_dtype)
            db = db.to(ctx.w_dtype)
        return (dx, dx if ctx.has_res else None, dg if need_w else None, db if need_w else None,
                None)


def layer_norm(x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
               eps: float = 1e-5, residual: Optional[torch.Tensor] = None):
    """LayerNorm over the last dim. With ``residual`` returns ``(LN(x + residual), x + residual)``
    from one HBM pass (pre-LN transformer block pattern)."""
    if not _gpu_ok(x) or x.shape[-1] > 8192:
        return reference_layer_norm(x, weight, bias, eps, residual)
    return _LayerNorm.apply(x, residual, weight, bias, eps)


def _bias_arg(bias: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    # the kernels read fp32 or bf16 biases directly; anything else is cast once
    if bias is None or (bias.dtype in (torch.float32, torch.bfloat16) and bias.is_contiguous()):
        return bias
    return bias.float().contiguous()


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        x = x.contiguous()
        b = _bias_arg(bias)
        y = _ext.load().bias_gelu(x, b)
        ctx.save_for_backward(x, b)
        ctx.bias = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        need_db = b is not None and ctx.needs_input_grad[1]
        acc = _grad.target(ctx.bias) if need_db else None
        dx, db = _ext.load().bias_gelu_bwd(dy, x, b, need_db, acc)
        if not need_db or acc is not None:
            return dx, None
        return dx, db.to(ctx.bias.dtype)


# K-slices of the split-K weight gradient (4 measured best: profiles/round5_gpt2_wgrad_splitk_ab.txt)
_WGRAD_SPLITS = 4
# linear-layer weight gradients on the side stream (ops/_grad.py); A/B switch
LINEAR_SIDE_STREAM = os.environ.get("DCA_LINEAR_WGRAD_STREAM", "1") != "0"


def _wgrad_splits(tokens: int, m: int, n: int) -> int:
    """Split-K factor for the weight gradient dW[m, n] = dY^T X over ``tokens``.

    A transformer's dW GEMMs have a small output (1-4M elements: 64-256 macro tiles for 256 CUs)
    and a long K (all tokens of the micro-batch), and hipBLASLt's heuristic runs them without
    split-K. Splitting K four ways as one batched GEMM fills the chip: measured on MI355X at 16k
    tokens (tools/bench_wgrad.py, profiles/r9_wgrad_splitk.txt) 1024x1024 111 -> 64 us,
    3072x1024 166 -> 115 us, 4096x1024 166 -> 145 us, 1024x4096 161 -> 143 us."""
    if tokens < 8192 or tokens % 4 or m * n > 16 * 2 ** 20:
        return 1
    if (m * n) % 8 or tokens % _WGRAD_SPLITS:  # splitk_accumulate: 8 elements per thread
        return 1
    return _WGRAD_SPLITS


def _wgrad_split_k(acc: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, s: int) -> None:
    """``acc += dy2^T x2`` as ``s`` K-slices in one batched GEMM with fp32 outputs, summed and
    added into ``acc`` by one fused kernel (``splitk_accumulate``: fixed-order fp32 sum of the
    slices, then the bf16/fp32 accumulate)."""
    t, m = dy2.shape
    a = dy2.reshape(s, t // s, m).transpose(1, 2)
    b = x2.reshape(s, t // s, x2.shape[1])
    _ext.load().splitk_accumulate(torch.bmm(a, b, out_dtype=torch.float32), acc)


def _weight_grad(w_param: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> Optional[torch.Tensor]:
    """dW = dy2^T x2, accumulated into the parameter's flat ``.grad`` view on the side stream
    (split-K batched GEMM at >= 8k tokens; returns None) or returned when there is no such view."""
    acc = _grad.target(w_param)
    if acc is None:
        return dy2.t() @ x2
    s = _wgrad_splits(dy2.shape[0], dy2.shape[1], x2.shape[1])
    side = _grad.side_stream_for(w_param) if LINEAR_SIDE_STREAM else None
    if side is not None:
        _grad.fork(side, (dy2, x2))
    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
        if s > 1:
            _wgrad_split_k(acc, dy2, x2, s)
        else:
            acc.addmm_(dy2.t(), x2)
    return None


def _bias_grad(b_param: torch.Tensor, dy2: torch.Tensor) -> Optional[torch.Tensor]:
    """db = dy2.sum(0): the fused column reduction straight into the flat ``.grad`` view (returns
    None) or a returned gradient."""
    acc = _grad.target(b_param)
    if dy2.shape[-1] % 8 == 0 and dy2.is_cuda:
        out = _ext.load().bias_grad(dy2, acc)
        return None if acc is not None else out.to(b_param.dtype)
    return dy2.sum(0).to(b_param.dtype)


class _Linear(torch.autograd.Function):
    """``y = x @ w.T + b`` whose backward accumulates straight into the parameters' flat
    ``.grad`` views: dW by a GEMM with beta = 1 (``grad.addmm_``), db by the fused column
    reduction (``bias_grad``) -- no AccumulateGrad adds, no torch reduce kernel (see
    ``ops._grad``). Falls back to returning gradients when the parameters have no persistent
    ``.grad``."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.params = (weight, bias)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        w_param, b_param = ctx.params
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[1]:  # first: on the side stream it overlaps the data gradient
            dw = _weight_grad(w_param, dy2, x.reshape(-1, x.shape[-1]))
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ weight).view(*dy.shape[:-1], weight.shape[1])
        given = getattr(ctx, "_dca_bias_given", None)
        if given is not None:
            ctx._dca_bias_given = None
            if dy.data_ptr() == given.data_ptr() and dy.shape == given.shape and dy.stride() == given.stride():
                return dx, dw, None  # bias gradient reduced by the consuming LayerNorm's backward
            # dy also carries gradient from another consumer: add only that part
            dy2 = (dy - given).reshape(-1, dy.shape[-1])
        if b_param is not None and ctx.needs_input_grad[2]:
            db = _bias_grad(b_param, dy2)
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.linear`` with fused gradient accumulation into flat ``.grad`` buffers on the GPU."""
    if not x.is_cuda or x.dtype != weight.dtype or (bias is not None and bias.dtype != x.dtype) or \
            torch.is_autocast_enabled():
        return F.linear(x, weight, bias)
    return _Linear.apply(x, weight, bias)


def bias_gelu(x: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """``gelu_tanh(x + bias)`` with the bias broadcast over the last dim."""
    if not _gpu_ok(x):
        return reference_bias_gelu(x, bias)
    return _BiasGelu.apply(x, bias)


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, rot):
        B, S, H, D = x.shape
        x = x.contiguous()
        ctx.save_for_backward(cos, sin)
        ctx.meta = (H, S, rot)
        return _ext.load().rope(x, cos, sin, H, S, rot, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        H, S, rot = ctx.meta
        return _ext.load().rope(dy.contiguous(), cos, sin, H, S, rot, True), None, None, None


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
         rot_dim: Optional[int] = None) -> torch.Tensor:
    """Rotary embedding (rotate-half convention) on the first ``rot_dim`` features of
    ``x`` [B, S, H, D]; ``cos``/``sin`` are [>=S, rot_dim/2] fp32 tables."""
    rot = rot_dim or x.shape[-1]
    if not _gpu_ok(x, 2):
        return reference_rope(x, cos, sin, rot)
    S = x.shape[1]
    half = rot // 2
    cos = cos[:S, :half].contiguous()
    sin = sin[:S, :half].contiguous()
    if cos.dtype != torch.float32:
        cos, sin = cos.float(), sin.float()
    return _Rope.apply(x, cos, sin, rot)


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, kv_len):
        o, lse = _ext.load().attn_fwd(q, k, v, scale, causal, kv_len)
        ctx.save_for_backward(q, k, v, o, lse, kv_len)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kv_len = ctx.saved_tensors
        dq, dk, dv = _ext.load().attn_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal, kv_len=kv_len)
        return dq, dk, dv, None, None, None


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        C = _ext.load()
        lse, loss_rows = C.ce_fwd(logits, target, ignore_index)
        n_valid = (target != ignore_index).sum().float()
        ctx.save_for_backward(logits, target, lse, n_valid)
        ctx.ignore_index = ignore_index
        return loss_rows.sum() / n_valid.clamp_min(1.0)

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, n_valid = ctx.saved_tensors
        gscale = torch.stack([g.float().reshape(()), n_valid]).contiguous()
        d = _ext.load().ce_bwd(logits, target, lse, gscale, ctx.ignore_index)
        return d, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy over rows of ``logits`` [..., V] without materialising fp32
    logits or log-probabilities: one read forward, one read + one write backward."""
    V = logits.shape[-1]
    l2 = logits.reshape(-1, V)
    t = target.reshape(-1)
    if not (logits.is_cuda and V % 8 == 0 and logits.dtype in (torch.bfloat16, torch.float16, torch.float32)):
        return F.cross_entropy(l2.float(), t, ignore_index=ignore_index)
    return _CrossEntropy.apply(l2.contiguous(), t.contiguous().long(), ignore_index)


class _FlashAttentionQKVPacked(torch.autograd.Function):
    """Attention on a fused QKV projection output [B, S, 3, H, D]: q/k/v are strided views and the
    backward writes dQ/dK/dV straight into one packed gradient (no stack/cat)."""

    @staticmethod
    def forward(ctx, qkv, causal, scale, kv_len):
        q, k, v = qkv.unbind(2)
        o, lse = _ext.load().attn_fwd(q, k, v, scale, causal, kv_len)
        ctx.save_for_backward(qkv, o, lse, kv_len)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kv_len = ctx.saved_tensors
        q, k, v = qkv.unbind(2)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.unbind(2)
        _ext.load().attn_bwd(do, q, k, v, o, lse, ctx.scale, ctx.causal, dq, dk, dv, kv_len)
        return dqkv, None, None, None


def _kv_len(key_lengths: Optional[torch.Tensor], B: int, device) -> Optional[torch.Tensor]:
    if key_lengths is None:
        return None
    if key_lengths.numel() != B:
        raise ValueError(f"key_lengths must have one entry per batch row ({B})")
    return key_lengths.to(device=device, dtype=torch.int32).contiguous()


def flash_attention_qkvpacked(qkv: torch.Tensor, causal: bool = True,
                              scale: Optional[float] = None,
                              key_lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``flash_attention`` for a packed [B, S, 3, H, D] QKV tensor -> [B, S, H, D]."""
    scale = scale if scale is not None else 1.0 / math.sqrt(qkv.shape[-1])
    q, k, v = qkv.unbind(2)
    if not qkv.is_cuda:
        return reference_attention(q, k, v, causal, scale, key_lengths)
    if not _attn_gpu_ok(q, k, v):
        raise ValueError("flash_attention_qkvpacked: GPU path needs bf16 [B,S,3,H,D] with D in "
                         "{64,128} and 16-byte aligned rows")
    return _FlashAttentionQKVPacked.apply(qkv, causal, float(scale),
                                          _kv_len(key_lengths, qkv.shape[0], qkv.device))


def _attn_gpu_ok(q, k, v) -> bool:
    if not (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128)):
        return False
    if k.shape != v.shape or k.shape[2] == 0 or q.shape[2] % k.shape[2]:
        return False
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
            return False
    return True


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: Optional[float] = None,
                    key_lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """softmax(q k^T * scale [+ causal mask] [+ key padding]) v for [B, S, H, Dh] operands (Dh in
    {64, 128}, bf16 on GPU). k / v may have fewer heads Hkv dividing H (grouped-query / multi-query
    attention: H / Hkv consecutive query heads share a K/V head; dK / dV sum over the group inside
    the kernel). Never materialises the S x S score matrix. ``key_lengths`` [B]
    (any integer dtype) is the number of valid keys per batch row -- right-padded batches such as
    an HF ``attention_mask``; padded keys get zero weight and zero dK/dV, and every query row
    (padded ones too) attends to the valid keys, as with an additive padding mask."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if not q.is_cuda:
        return reference_attention(q, k, v, causal, scale, key_lengths)
    if not _attn_gpu_ok(q, k, v):
        raise ValueError("flash_attention: GPU path needs bf16 [B,S,H,D] with D in {64,128}, "
                         "K/V heads dividing the query heads and 16-byte aligned rows")
    return _FlashAttention.apply(q, k, v, causal, float(scale), _kv_len(key_lengths, q.shape[0], q.device))


__all__ = ["layer_norm", "bias_gelu", "rope", "rope_tables", "flash_attention",
           "flash_attention_qkvpacked", "cross_entropy",
           "reference_layer_norm", "reference_bias_gelu", "reference_rope", "reference_attention"]
