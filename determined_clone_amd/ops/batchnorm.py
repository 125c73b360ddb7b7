"""Fused BatchNorm(+residual)(+ReLU) op.

GPU path: `ops/csrc/batchnorm.hip` (NHWC, 2 HBM passes forward, 2 backward).
CPU path: the plain PyTorch reference (`F.batch_norm` + add + relu) used by CPU tests and as the
fp32 oracle for the GPU numerics tests.
"""
from typing import Optional

import torch
import torch.nn.functional as F

from determined_clone_amd.ops import _ext, _grad


def reference_batch_norm_act(x, weight, bias, running_mean, running_var, residual=None,
                             training=True, momentum=0.1, eps=1e-5, relu=True):
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class ResidualGradSink:
    """Mailbox for the gradient of a fused-BN output that another fused BN consumes as its
    residual. The consumer deposits d(residual) here instead of returning it to autograd, and the
    producer's backward adds it inside its own kernels (dy + dy2) -- this removes the separate
    full-tensor add autograd would otherwise run for every identity shortcut of a ResNet.
    Ordering is guaranteed by the data flow: the consumer's backward precedes the backward of the
    producer's other consumers (conv1 of the same block), which the producer waits for."""

    __slots__ = ("grad",)

    def __init__(self) -> None:
        self.grad: Optional[torch.Tensor] = None

    def deposit(self, g: torch.Tensor) -> None:
        self.grad = g if self.grad is None else self.grad + g


class _BNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, num_batches, momentum,
                eps, relu, res_sink, out_sink, partials):
        C = _ext.load()
        y, mean, invstd, mask = C.bn_fwd_train(x, residual, weight, bias, running_mean,
                                               running_var, num_batches, momentum, eps, relu,
                                               partials)
        # The ReLU decision is kept as a bitmask (1/16 of y) instead of y itself.
        ctx.save_for_backward(x, mask if relu else None, weight, mean, invstd)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.res_sink = res_sink      # where to deposit d(residual) (or None: return it)
        ctx.out_sink = out_sink      # extra upstream gradient of y deposited by a consumer
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd = ctx.saved_tensors
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dy2 = ctx.out_sink.grad if ctx.out_sink is not None else None
        if ctx.out_sink is not None:
            ctx.out_sink.grad = None
        acc_w, acc_b = _direct_grad_targets(*ctx.params) if need_w else (None, None)
        dx, dgamma, dbeta, dres = _ext.load().bn_bwd_train(
            dy, x, mask, weight, mean, invstd, ctx.relu, ctx.has_res, need_w, dy2, acc_w, acc_b)
        if acc_w is not None:
            need_w = False  # already accumulated into .grad by the finalize kernel
        dres_out = None
        if ctx.has_res:
            if ctx.res_sink is not None:
                ctx.res_sink.deposit(dres)
            else:
                dres_out = dres
        return (dx, dgamma if need_w else None, dbeta if need_w else None, dres_out,
                None, None, None, None, None, None, None, None, None)


def _direct_grad_targets(weight: Optional[torch.Tensor], bias: Optional[torch.Tensor]):
    """``(weight.grad, bias.grad)`` when the BN finalize kernel may accumulate dgamma/dbeta into
    them directly (see ``ops._grad``), else ``(None, None)``."""
    gw, gb = _grad.target(weight), _grad.target(bias)
    if gw is None or gb is None or gw.dtype != torch.float32 or gb.dtype != torch.float32:
        return None, None
    return gw, gb


def _hip_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dim() not in (2, 4) or x.size(1) % 8 != 0:
        return False
    return x.dtype in (torch.bfloat16, torch.float16, torch.float32)


def batch_norm_act(x: torch.Tensor, weight: Optional[torch.Tensor], bias: Optional[torch.Tensor],
                   running_mean: Optional[torch.Tensor], running_var: Optional[torch.Tensor],
                   residual: Optional[torch.Tensor] = None, training: bool = True,
                   momentum: Optional[float] = 0.1, eps: float = 1e-5, relu: bool = True,
                   num_batches_tracked: Optional[torch.Tensor] = None,
                   fuse_residual_grad: bool = False) -> torch.Tensor:
    """``act(batch_norm(x) + residual)`` with torch BatchNorm semantics (biased variance for the
    normalisation, unbiased for the running estimate).

    ``fuse_residual_grad=True`` (caller guarantees that ``residual`` -- if it is the output of
    another fused BN -- is ALSO consumed by an autograd op that runs after this op's backward, e.g.
    the identity shortcut of a ResNet block whose input also feeds conv1): the residual gradient is
    handed to the producer through a :class:`ResidualGradSink` and summed inside its backward
    kernels instead of by a separate autograd add."""
    if not _hip_ok(x) or momentum is None:
        if momentum is None and training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
            momentum = 1.0 / float(num_batches_tracked.item())
        elif training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        return reference_batch_norm_act(x, weight, bias, running_mean, running_var, residual,
                                        training, momentum if momentum is not None else 0.0, eps,
                                        relu)
    # per-block (sum, sum^2) of x already reduced by its producer (ops.conv.pointwise_conv)
    partials = getattr(x, "_dca_bn_partials", None)
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
        # Residual produced by another fused BN (identity shortcut): route its gradient through a
        # sink so the producer sums it in-kernel instead of autograd running a separate add.
        res_sink = None
        if fuse_residual_grad and residual is not None and residual.requires_grad and torch.is_grad_enabled():
            res_sink = getattr(residual, "_dca_grad_sink", None)
            if res_sink is not None:
                residual = residual.detach()
        out_sink = ResidualGradSink() if torch.is_grad_enabled() else None
        y = _BNActTrain.apply(x, weight, bias, residual,
                                 running_mean if training else None,
                                 running_var if training else None,
                                 num_batches_tracked if training else None, float(momentum),
                                 float(eps), relu, res_sink, out_sink, partials)
        if out_sink is not None:
            y._dca_grad_sink = out_sink
        return y
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


# ----------------------------------------------------------------------------- stem fusion
def reference_bn_relu_maxpool(x, weight, bias, running_mean, running_var, training=True,
                              momentum=0.1, eps=1e-5):
    y = F.relu(F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps))
    return F.max_pool2d(y, 3, 2, 1)


class _BNReLUPoolTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, num_batches, momentum, eps):
        y, mean, invstd, idx = _ext.load().bn_pool_fwd_train(x, weight, bias, running_mean,
                                                             running_var, num_batches, momentum, eps)
        ctx.save_for_backward(x, idx, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, weight, mean, invstd = ctx.saved_tensors
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dx, dg, db = _ext.load().bn_pool_bwd(dy, x, idx, weight, mean, invstd, need_w)
        return dx, dg if need_w else None, db if need_w else None, None, None, None, None, None


def batch_norm_relu_maxpool(x: torch.Tensor, weight: Optional[torch.Tensor],
                            bias: Optional[torch.Tensor], running_mean: Optional[torch.Tensor],
                            running_var: Optional[torch.Tensor], training: bool = True,
                            momentum: Optional[float] = 0.1, eps: float = 1e-5,
                            num_batches_tracked: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``max_pool2d(relu(batch_norm(x)), 3, 2, 1)`` -- the ResNet stem -- without writing the
    pre-pool activation; backward gathers the pooled gradient inside the BN-backward passes."""
    if not (_hip_ok(x) and x.dim() == 4) or momentum is None:
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
            if momentum is None:
                momentum = 1.0 / float(num_batches_tracked.item())
        return reference_bn_relu_maxpool(x, weight, bias, running_mean, running_var, training,
                                         momentum if momentum is not None else 0.0, eps)
    x = x.contiguous(memory_format=torch.channels_last)
    if training or running_mean is None:
        return _BNReLUPoolTrain.apply(x, weight, bias, running_mean if training else None,
                                      running_var if training else None,
                                      num_batches_tracked if training else None, float(momentum),
                                      float(eps))
    scale = torch.rsqrt(running_var.float() + eps)
    if weight is not None:
        scale = scale * weight.float()
    shift = -running_mean.float() * scale
    if bias is not None:
        shift = shift + bias.float()
    if torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)):
        shape = (1, -1, 1, 1)
        y = F.relu(x * scale.view(shape).to(x.dtype) + shift.view(shape).to(x.dtype))
        return F.max_pool2d(y, 3, 2, 1)
    return _ext.load().bn_pool_fwd_affine(x, scale, shift)


# ----------------------------------------------------------------------------- global avg pool
class _SpatialMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, g):
        return _ext.load().spatial_mean_bwd(g, *ctx.hw)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``flatten(adaptive_avg_pool2d(x, 1), 1)`` for an NHWC activation; on the GPU the backward
    broadcast g / (H*W) is one streaming kernel (``csrc/batchnorm.hip``)."""
    if _hip_ok(x) and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return _SpatialMean.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
