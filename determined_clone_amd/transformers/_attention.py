"""Hugging Face attention backend on the framework's flash-attention kernels.

``use_flash_attention(model)`` switches a ``transformers`` model (BERT, RoBERTa, ViT, GPT-2, ...
anything that dispatches through ``ALL_ATTENTION_FUNCTIONS``) to ``"dca_mfma"``: q/k/v arrive as
[B, H, S, D] views and go to ``ops.transformer.flash_attention`` as [B, S, H, D] strided views
(no copies). A padding ``attention_mask`` -- the boolean [B, 1, Sq, Sk] mask HF builds from a
right-padded ``attention_mask`` -- becomes per-row key lengths for the kernels' key-padding path,
so padded BERT batches never materialise scores either. Anything else falls back to HF's SDPA
path: masks that are not right padding (left padding, packed sequences, custom masks), attention
dropout in training, grouped KV heads, head dims other than 64/128, non-bf16 or CPU tensors.

The reference trains HF models through its Trainer callback (harness/determined/transformers/
_hf_callback.py) on the stock CUDA attention; this module is the MI355X-side kernel hookup.
"""
import weakref
from typing import Any, Optional, Tuple

import torch

from determined_clone_amd.ops import transformer as T

NAME = "dca_mfma"  # (HF treats names containing "flash" as flash-attn kernels)

# HF hands the same mask object to every layer of one forward: convert it once
_cache: Tuple[Any, ...] = (None, -1, None, None)


def mask_to_key_lengths(mask: torch.Tensor, causal: bool) -> Optional[torch.Tensor]:
    """Boolean [B, 1|H, Sq, Sk] mask (True = attend) -> int32 key lengths [B], or None when the
    mask is not pure right padding (optionally combined with the causal triangle)."""
    global _cache
    ref, ver, cz, out = _cache
    if ref is not None and ref() is mask and ver == mask._version and cz == causal:
        return out
    res: Optional[torch.Tensor] = None
    if mask.dtype == torch.bool and mask.dim() == 4:
        B, _, Sq, Sk = mask.shape
        last = mask[:, 0, -1, :]  # the last query row sees every valid key (causal or not)
        lengths = last.sum(-1)
        keys = torch.arange(Sk, device=mask.device)
        want = (keys[None, :] < lengths[:, None])[:, None, None, :]
        if causal:
            want = want & torch.ones(Sq, Sk, dtype=torch.bool, device=mask.device).tril(Sk - Sq)
        ok = bool(torch.equal(mask, want.expand_as(mask))) and bool((lengths > 0).all())
        res = lengths.to(torch.int32) if ok else None
    _cache = (weakref.ref(mask), mask._version, causal, res)
    return res


def _sdpa(*args: Any, **kwargs: Any) -> Any:
    from transformers.integrations.sdpa_attention import sdpa_attention_forward

    return sdpa_attention_forward(*args, **kwargs)


def flash_attention_forward(module: torch.nn.Module, query: torch.Tensor, key: torch.Tensor,
                            value: torch.Tensor, attention_mask: Optional[torch.Tensor],
                            scaling: Optional[float] = None, dropout: float = 0.0,
                            **kwargs: Any) -> Tuple[torch.Tensor, None]:
    """The ``AttentionInterface`` callable: returns ([B, S, H, D], None)."""
    causal = bool(kwargs.get("is_causal", getattr(module, "is_causal", False)))
    Sq, Sk = query.shape[2], key.shape[2]
    usable = (query.is_cuda and query.dtype == torch.bfloat16 and query.shape[-1] in (64, 128)
              and query.shape[1] % key.shape[1] == 0 and not (dropout > 0 and module.training)
              and (not causal or Sq == Sk))
    kv_len = None
    if usable and attention_mask is not None:
        kv_len = mask_to_key_lengths(attention_mask, causal)
        usable = kv_len is not None
    q, k, v = (t.transpose(1, 2) for t in (query, key, value))
    if not (usable and T._attn_gpu_ok(q, k, v)):
        return _sdpa(module, query, key, value, attention_mask, scaling=scaling, dropout=dropout,
                     **kwargs)
    return T.flash_attention(q, k, v, causal=causal, scale=scaling, key_lengths=kv_len), None


def register() -> str:
    """Register ``"dca_mfma"`` with HF's attention and mask interfaces (idempotent)."""
    from transformers import AttentionInterface, AttentionMaskInterface
    from transformers.masking_utils import sdpa_mask

    AttentionInterface.register(NAME, flash_attention_forward)
    AttentionMaskInterface.register(NAME, sdpa_mask)  # boolean masks, None when nothing is masked
    return NAME


def use_flash_attention(model: Any) -> Any:
    """Switch ``model`` (a ``transformers.PreTrainedModel``) to the flash-attention kernels."""
    model.set_attn_implementation(register())
    return model
