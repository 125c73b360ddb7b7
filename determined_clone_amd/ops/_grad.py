"""In-kernel gradient accumulation into parameters' persistent ``.grad`` views.

The framework keeps every trainable parameter's gradient in a flat buffer
(``parallel.flat.FlatParamSpace``, used by the fused optimizers, the bucketed RCCL all-reduce and
ZeRO). Those ``.grad`` tensors never change identity, so a backward kernel can ADD its result
straight into them: the BN / LayerNorm / bias column reductions store with ``+=`` in their final
pass, and a linear layer's weight gradient is a GEMM with beta = 1 on the ``.grad`` view. The
op's autograd backward then returns None for that parameter. Autograd's AccumulateGrad node still
runs -- with an undefined gradient it launches nothing -- and still calls the parameter's
post-accumulate hooks, which the gradient-sync buckets count. Kernels run on the current stream
in backward order, so the hooks see the gradient "ready" exactly as before.

This removes one elementwise add kernel per parameter per backward (about 290 launches per
GPT-2-medium step -- linear weights/biases and LayerNorm affine -- and 106 per ResNet-50 step, the
BatchNorm affine parameters). The same idea appears as Megatron-LM's
"gradient accumulation fusion". ``DCA_DIRECT_GRAD=0`` turns it off.

Caveat: ``torch.autograd.grad(...)`` over such parameters would also accumulate into ``.grad``,
because a backward pass cannot tell it is being driven by ``autograd.grad``. Call
``FlatParamSpace.release_direct_grad()`` (or set ``DCA_DIRECT_GRAD=0``) for that pattern.
"""
import os
from typing import Optional

import torch

ENABLED = os.environ.get("DCA_DIRECT_GRAD", "1") != "0"


def target(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The ``.grad`` tensor a kernel may accumulate into for parameter ``p``, or None."""
    if not ENABLED or p is None or not getattr(p, "_dca_direct_grad", False):
        return None
    g = p.grad
    if g is None or g.dtype != p.dtype or not g.is_contiguous() or g.shape != p.shape:
        return None
    if g.dtype not in (torch.float32, torch.bfloat16):
        return None
    return g
