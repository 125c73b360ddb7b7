"""Fused BatchNorm(+residual)(+ReLU) op.

GPU path: `ops/csrc/batchnorm.hip` (NHWC, 2 HBM passes forward, 2 backward).
CPU path: the plain PyTorch reference (`F.batch_norm` + add + relu) used by CPU tests and as the
fp32 oracle for the GPU numerics tests.
"""
from typing import Optional

import torch
import torch.nn.functional as F

from determined_clone_amd.ops import _ext


def reference_batch_norm_act(x, weight, bias, running_mean, running_var, residual=None,
                             training=True, momentum=0.1, eps=1e-5, relu=True):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, num_batches, momentum,
                eps, relu):
        C = _ext.load()
        y, mean, invstd, mask = C.bn_fwd_train(x, residual, weight, bias, running_mean,
                                               running_var, num_batches, momentum, eps, relu)
        # The ReLU decision is kept as a bitmask (1/16 of y) instead of y itself.
        ctx.save_for_backward(x, mask if relu else None, weight, mean, invstd)
        ctx.relu = relu
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dx, dgamma, dbeta, dres = _ext.load().bn_bwd_train(
            dy, x, mask, weight, mean, invstd, ctx.relu, ctx.has_res, need_w)
        return (dx, dgamma if need_w else None, dbeta if need_w else None,
                dres if ctx.has_res else None, None, None, None, None, None, None)


def _hip_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dim() not in (2, 4) or x.size(1) % 8 != 0:
        return False
    return x.dtype in (torch.bfloat16, torch.float16, torch.float32)


def batch_norm_act(x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
                   running_mean: Optional[torch.Tensor], running_var: Optional[torch.Tensor],
                   residual: Optional[torch.Tensor] = None, training: bool = True,
                   momentum: Optional[float] = 0.1, eps: float = 1e-5, relu: bool = True,
                   num_batches_tracked: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``act(batch_norm(x) + residual)`` with torch BatchNorm semantics (biased variance for the
    normalisation, unbiased for the running estimate)."""
    if not _hip_ok(x) or momentum is None:
        if momentum is None and training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
            momentum = 1.0 / float(num_batches_tracked.item())
        elif training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        return reference_batch_norm_act(x, weight, bias, running_mean, running_var, residual,
                                        training, momentum if momentum is not None else 0.0, eps,
                                        relu)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
        if residual is not None:
            residual = residual.contiguous(memory_format=torch.channels_last)
    else:
        x = x.contiguous()
        residual = residual.contiguous() if residual is not None else None
    if residual is not None and residual.dtype != x.dtype:
        residual = residual.to(x.dtype)
    use_batch_stats = training or running_mean is None
    if use_batch_stats:
        return _BNActTrain.apply(x, weight, bias, residual,
                                 running_mean if training else None,
                                 running_var if training else None,
                                 num_batches_tracked if training else None, float(momentum),
                                 float(eps), relu)
    # Inference: per-channel affine from the running statistics.
    scale = torch.rsqrt(running_var.float() + eps)
    if weight is not None:
        scale = scale * weight.float()
    shift = -running_mean.float() * scale
    if bias is not None:
        shift = shift + bias.float()
    if torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)):
        shape = (1, -1) + (1,) * (x.dim() - 2)
        y = x * scale.view(shape).to(x.dtype) + shift.view(shape).to(x.dtype)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
    return _ext.load().bn_fwd_affine(x, residual, scale, shift, relu)
