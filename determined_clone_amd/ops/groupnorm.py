"""NHWC GroupNorm (+ fused SiLU) on the HIP kernels of ``csrc/groupnorm.hip``.

GPU path: bf16/fp32 channels_last activations, fp32 affine parameters; the forward saves only
per-(sample, channel) fp32 coefficients (no normalised copy), the backward recomputes the
pre-activation and accumulates dgamma/dbeta straight into the parameters' persistent ``.grad``
views when the optimizer's flat buffers own them (``ops/_grad.py``). CPU / other layouts:
``torch.nn.functional.group_norm`` (+ ``silu``), also the fp32 oracle of the GPU tests.
"""
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import _ext, _grad


class _GroupNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, act):
        y, scale, shift, xa, xb, mean, rstd = _ext.load().gn_fwd(x, weight, bias, groups, eps, act)
        ctx.save_for_backward(x, weight, bias, scale, shift, xa, xb, mean, rstd)
        ctx.groups, ctx.act = groups, act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, scale, shift, xa, xb, mean, rstd = ctx.saved_tensors
        need = w is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        acc_w, acc_b = (_grad.target(w), _grad.target(b)) if need else (None, None)
        if acc_w is None or acc_b is None or acc_w.dtype != torch.float32 or acc_b.dtype != torch.float32:
            acc_w = acc_b = None
        dx, dw, db = _ext.load().gn_bwd(dy, x, w, scale, shift, xa, xb, mean, rstd, ctx.groups,
                                        ctx.act, need, acc_w, acc_b)
        if acc_w is not None:
            dw = db = None  # accumulated into the persistent .grad views in-kernel
        return dx, dw, db, None, None, None




def _gpu_ok(x: torch.Tensor, weight: Optional[torch.Tensor], groups: int) -> bool:
    if not x.is_cuda or x.dim() != 4 or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    C = x.shape[1]
    if C % 8 or C % groups or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    return weight is None or (weight.dtype == torch.float32 and weight.is_contiguous())


def group_norm_act(x: torch.Tensor, groups: int, weight: Optional[torch.Tensor] = None,
                   bias: Optional[torch.Tensor] = None, eps: float = 1e-5, act: bool = False) -> torch.Tensor:
    """``silu(group_norm(x))`` (``act``) or ``group_norm(x)``."""
    if _gpu_ok(x, weight, groups):
        return _GroupNormAct.apply(x, weight, bias, groups, float(eps), bool(act))
    y = F.group_norm(x, groups, None if weight is None else weight.to(x.dtype),
                     None if bias is None else bias.to(x.dtype), eps)
    return F.silu(y) if act else y


class GroupNormAct(nn.GroupNorm):
    """``nn.GroupNorm`` with an optional fused SiLU; same parameter names (checkpoints
    interchange). Affine parameters are kept fp32 by :meth:`_apply` overrides in the model's
    ``to_mi355x_layout``."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-5, act: bool = False) -> None:
        super().__init__(num_groups, num_channels, eps)
        self.act = act

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return group_norm_act(x, self.num_groups, self.weight, self.bias, self.eps, self.act)
