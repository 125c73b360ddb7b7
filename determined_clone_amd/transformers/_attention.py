"""Hugging Face attention backend on the framework's flash-attention kernels.

``use_flash_attention(model)`` switches a ``transformers`` model (BERT, RoBERTa, ViT, GPT-2, ...
anything that dispatches through ``ALL_ATTENTION_FUNCTIONS``) to ``"dca_mfma"``: q/k/v arrive as
[B, H, S, D] views and go to ``ops.transformer.flash_attention`` as [B, S, H, D] strided views
(no copies). A padding ``attention_mask`` -- the boolean [B, 1, Sq, Sk] mask HF builds from a
right-padded ``attention_mask`` -- becomes per-row key lengths for the kernels' key-padding path,
so padded BERT batches never materialise scores either. The lengths are derived from the 2-D
``attention_mask`` HF passes to the mask interface (one small [B, Sk] check per distinct mask
object, cached by object and version, so a reused mask costs no host sync) and ride on the 4-D
mask to the layers. Grouped KV heads (GQA / MQA, ``H % Hkv == 0``) run natively in the kernels.
Anything else falls back to HF's SDPA path: masks that are not right padding (left padding,
packed sequences, sliding windows, custom masks), attention dropout in training, head dims other
than 64/128, non-bf16 or CPU tensors.

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
    mask is not pure right padding (optionally combined with the causal triangle). A mask built by
    this backend's mask function carries its lengths (no device check here); other masks are
    compared against the padding pattern once per mask object."""
    got = getattr(mask, "_dca_key_lengths", None)
    if got is not None and getattr(mask, "_dca_causal", None) == causal:
        return got if isinstance(got, torch.Tensor) else None
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


# 2-D padding mask -> lengths (or False: not right padding), keyed by object and version
_lengths_cache: Tuple[Any, ...] = (None, -1, None)


def padding_lengths(mask2d: torch.Tensor) -> Optional[torch.Tensor]:
    """int32 key lengths [B] of a 2-D right-padding ``attention_mask`` [B, Sk] (1 = token), or
    None when it is not right padding / a row is empty. One host sync on the small 2-D mask per
    distinct mask (object, version)."""
    global _lengths_cache
    ref, ver, out = _lengths_cache
    if ref is not None and ref() is mask2d and ver == mask2d._version:
        return out if isinstance(out, torch.Tensor) else None
    m = mask2d.bool()
    lengths = m.sum(-1)
    keys = torch.arange(m.shape[-1], device=m.device)
    ok = torch.logical_and((m == (keys[None, :] < lengths[:, None])).all(), (lengths > 0).all())
    res = lengths.to(torch.int32) if bool(ok) else False
    _lengths_cache = (weakref.ref(mask2d), mask2d._version, res)
    return res if isinstance(res, torch.Tensor) else None


def _mask(*args: Any, **kwargs: Any) -> Optional[torch.Tensor]:
    """HF mask-interface function: ``sdpa_mask`` (boolean 4-D masks, None when nothing is masked)
    that also attaches the key lengths of a right-padding ``attention_mask`` to the mask it
    returns, when the rest of the mask is the plain causal or bidirectional pattern."""
    from transformers import masking_utils as mu

    out = mu.sdpa_mask(*args, **kwargs)
    mask2d = kwargs.get("attention_mask")
    fn = kwargs.get("mask_function", mu.causal_mask_function)
    causal = {mu.causal_mask_function: True,
              getattr(mu, "bidirectional_mask_function", None): False}.get(fn)
    if (isinstance(out, torch.Tensor) and isinstance(mask2d, torch.Tensor) and mask2d.dim() == 2
            and causal is not None and kwargs.get("local_size") is None
            and not kwargs.get("q_offset") and not kwargs.get("kv_offset")
            and mask2d.shape[-1] == out.shape[-1]):
        lengths = padding_lengths(mask2d)
        out._dca_key_lengths = lengths if lengths is not None else False
        out._dca_causal = causal
    return out


def register() -> str:
    """Register ``"dca_mfma"`` with HF's attention and mask interfaces (idempotent)."""
    from transformers import AttentionInterface, AttentionMaskInterface

    AttentionInterface.register(NAME, flash_attention_forward)
    AttentionMaskInterface.register(NAME, _mask)
    return NAME


def use_flash_attention(model: Any) -> Any:
    """Switch ``model`` (a ``transformers.PreTrainedModel``) to the flash-attention kernels."""
    model.set_attn_implementation(register())
    return model
