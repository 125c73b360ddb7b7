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
            dy, x, mask, weight, mean, invstd, ctx.relu, ctx.has_res, need_w, dy2, acc_w, acc_b,
            None)
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


# ----------------------------------------------------------------------------- dual (shortcut) fusion
def _effective_momentum(m) -> float:
    """torch's BatchNorm momentum: ``momentum``, or with ``momentum=None`` the cumulative average
    1 / num_batches_tracked (read after this step's increment)."""
    if m.momentum is not None:
        return m.momentum
    if m.training and m.num_batches_tracked is not None:
        return 1.0 / float(m.num_batches_tracked.item())
    return 0.0


def reference_batch_norm_act_dual(x, bn, x2, bn2, relu=True):
    """fp32 / CPU oracle: ``act(bn(x) + bn2(x2))`` with two ``nn.BatchNorm2d``-like modules (their
    ``num_batches_tracked`` already advanced for this step when ``momentum`` is None)."""
    y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                     _effective_momentum(bn), bn.eps)
    y2 = F.batch_norm(x2, bn2.running_mean, bn2.running_var, bn2.weight, bn2.bias, bn2.training,
                      _effective_momentum(bn2), bn2.eps)
    y = y + y2
    return F.relu(y) if relu else y


class _BNActDualTrain(torch.autograd.Function):
    """``act(bn(x) + bn2(x2))``: the main-branch BatchNorm of a downsampling ResNet block and its
    projection shortcut's BatchNorm in one apply pass forward (the shortcut's normalised tensor is
    never written) and one statistics + one apply pass backward (both inputs' gradients from the
    shared masked gradient) -- ``csrc/batchnorm.hip`` ``bn_*_train_dual``."""

    @staticmethod
    def forward(ctx, x, weight, bias, x2, weight2, bias2, running_mean, running_var, num_batches,
                running_mean2, running_var2, num_batches2, momentum, eps, relu, out_sink,
                partials, partials2):
        y, m1, i1, mask, m2, i2 = _ext.load().bn_fwd_train_dual(
            x, weight, bias, running_mean, running_var, num_batches, x2, weight2, bias2,
            running_mean2, running_var2, num_batches2, momentum, eps, relu, partials, partials2)
        ctx.save_for_backward(x, x2, mask if relu else None, weight, weight2, m1, i1, m2, i2)
        ctx.relu = relu
        ctx.out_sink = out_sink
        ctx.params = (weight, bias, weight2, bias2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, x2, mask, weight, weight2, m1, i1, m2, i2 = ctx.saved_tensors
        n = ctx.needs_input_grad
        need_w = any(n[i] for i in (1, 2, 4, 5))
        dy2 = ctx.out_sink.grad if ctx.out_sink is not None else None
        if ctx.out_sink is not None:
            ctx.out_sink.grad = None
        acc = []
        if need_w:
            t1, t2 = _direct_grad_targets(ctx.params[0], ctx.params[1])
            t3, t4 = _direct_grad_targets(ctx.params[2], ctx.params[3])
            if all(t is not None for t in (t1, t2, t3, t4)):
                acc = [t1, t2, t3, t4]
        dx, dx2, dg, db, dg2, db2 = _ext.load().bn_bwd_train_dual(
            dy, x, mask, weight, m1, i1, x2, weight2, m2, i2, ctx.relu, need_w, dy2, acc)
        if acc:
            dg = db = dg2 = db2 = None  # accumulated into the parameters' .grad views
        return (dx, dg if n[1] else None, db if n[2] else None, dx2, dg2 if n[4] else None,
                db2 if n[5] else None) + (None,) * 12


def batch_norm_act_dual(x: torch.Tensor, bn: torch.nn.BatchNorm2d, x2: torch.Tensor,
                        bn2: torch.nn.BatchNorm2d, relu: bool = True) -> torch.Tensor:
    """``act(bn(x) + bn2(x2))`` -- e.g. ``relu(bn3(conv3(...)) + bn_ds(conv_ds(x)))``, a ResNet
    downsampling block's tail, with torch BatchNorm semantics for both (running statistics,
    ``num_batches_tracked``). GPU: fused kernels (see :class:`_BNActDualTrain`); the statistics
    partials a convolution epilogue attached to ``x`` / ``x2`` are used. Elsewhere: the plain
    PyTorch composition."""
    training = bn.training or bn.running_mean is None
    ok = (_hip_ok(x) and x.dim() == 4 and x2.shape == x.shape and x2.dtype == x.dtype
          and bn.momentum is not None and bn2.momentum is not None and training == (bn2.training or bn2.running_mean is None)
          and bn.eps == bn2.eps and bn.momentum == bn2.momentum)
    if not ok:
        for m in (bn, bn2):
            if m.training and m.num_batches_tracked is not None:
                m.num_batches_tracked.add_(1)
        return reference_batch_norm_act_dual(x, bn, x2, bn2, relu)
    p1 = getattr(x, "_dca_bn_partials", None)
    p2 = getattr(x2, "_dca_bn_partials", None)
    x = x.contiguous(memory_format=torch.channels_last)
    x2 = x2.contiguous(memory_format=torch.channels_last)
    if not training:  # inference: y = act(x*s + t + x2*s2 + t2)
        def affine(m):
            scale = torch.rsqrt(m.running_var.float() + m.eps)
            if m.weight is not None:
                scale = scale * m.weight.float()
            shift = -m.running_mean.float() * scale
            if m.bias is not None:
                shift = shift + m.bias.float()
            return scale, shift
        (s1, t1), (s2, t2) = affine(bn), affine(bn2)
        if torch.is_grad_enabled() and (x.requires_grad or x2.requires_grad):
            shape = (1, -1, 1, 1)
            y = x * s1.view(shape).to(x.dtype) + t1.view(shape).to(x.dtype) + \
                x2 * s2.view(shape).to(x.dtype) + t2.view(shape).to(x.dtype)
            return F.relu(y) if relu else y
        C = _ext.load()
        return C.bn_fwd_affine(x, C.bn_fwd_affine(x2, None, s2, t2, False), s1, t1, relu)
    out_sink = ResidualGradSink() if torch.is_grad_enabled() else None
    y = _BNActDualTrain.apply(x, bn.weight, bn.bias, x2, bn2.weight, bn2.bias,
                              bn.running_mean if bn.training else None,
                              bn.running_var if bn.training else None,
                              bn.num_batches_tracked if bn.training else None,
                              bn2.running_mean if bn2.training else None,
                              bn2.running_var if bn2.training else None,
                              bn2.num_batches_tracked if bn2.training else None,
                              float(bn.momentum), float(bn.eps), relu, out_sink, p1, p2)
    if out_sink is not None:
        y._dca_grad_sink = out_sink
    return y


# ----------------------------------------------------------------------------- stem fusion
def reference_bn_relu_maxpool(x, weight, bias, running_mean, running_var, training=True,
                              momentum=0.1, eps=1e-5):
    y = F.relu(F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps))
    return F.max_pool2d(y, 3, 2, 1)


class _BNReLUPoolTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, num_batches, momentum, eps,
                partials=None):
        y, mean, invstd, idx = _ext.load().bn_pool_fwd_train(x, weight, bias, running_mean,
                                                             running_var, num_batches, momentum, eps,
                                                             partials)
        ctx.save_for_backward(x, idx, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, weight, mean, invstd = ctx.saved_tensors
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dx, dg, db = _ext.load().bn_pool_bwd(dy, x, idx, weight, mean, invstd, need_w)
        return dx, dg if need_w else None, db if need_w else None, None, None, None, None, None, None


def batch_norm_relu_maxpool(x: torch.Tensor, weight: Optional[torch.Tensor],
                            bias: Optional[torch.Tensor], running_mean: Optional[torch.Tensor],
                            running_var: Optional[torch.Tensor], training: bool = True,
                            momentum: Optional[float] = 0.1, eps: float = 1e-5,
                            num_batches_tracked: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``max_pool2d(relu(batch_norm(x)), 3, 2, 1)`` -- the ResNet stem -- without writing the
    pre-pool activation; backward gathers the pooled gradient inside the BN-backward passes.
    Training statistics come from ``x._dca_bn_partials`` when the stem convolution's epilogue
    reduced them (``ops.conv.stem_conv(..., bn_stats=True)``)."""
    partials = getattr(x, "_dca_bn_partials", None)
    if not (_hip_ok(x) and x.dim() == 4) or momentum is None:
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
            if momentum is None:
                momentum = 1.0 / float(num_batches_tracked.item())
        return reference_bn_relu_maxpool(x, weight, bias, running_mean, running_var, training,
                                         momentum if momentum is not None else 0.0, eps)
    if not x.is_contiguous(memory_format=torch.channels_last):
        x, partials = x.contiguous(memory_format=torch.channels_last), None
    if training or running_mean is None:
        return _BNReLUPoolTrain.apply(x, weight, bias, running_mean if training else None,
                                      running_var if training else None,
                                      num_batches_tracked if training else None, float(momentum),
                                      float(eps), partials)
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
