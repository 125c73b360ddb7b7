"""Flat parameter / gradient spaces.

The reference keeps every parameter and gradient as a separate tensor and lets Horovod / torch DDP
copy them into fusion buffers each step (reference: `harness/determined/pytorch/_pytorch_context.py`
wrap_model / `_average_gradients`, Horovod `tensor_fusion_threshold`). On MI355X we instead lay
each optimizer's parameters out ONCE in flat per-dtype buffers and make ``p.data`` / ``p.grad``
views into them:

* the optimizer step is a single streaming HIP kernel per (dtype buffer, param group)
  (`ops/csrc/optim.hip`), not a loop over ~160 tensors;
* DDP buckets (`parallel/ddp.py`) are contiguous slices of the gradient buffer, all-reduced in
  place by RCCL with zero packing copies;
* ZeRO shards (`parallel/zero.py`) are per-bucket contiguous ranges of the same buffers
  (``pad_multiple`` pads each buffer to a whole number of world_size x ALIGN units).

Layout: params are grouped by dtype, then by optimizer param-group, and inside a group in REVERSE
registration order (the order autograd produces gradients), each segment padded to ``ALIGN``
elements so every view starts 128-byte aligned for 16-byte vector loads.
"""
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

ALIGN = 64  # elements; 128 B for bf16, 256 B for fp32


def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


def _dense_strides(p: torch.Tensor) -> bool:
    if p.is_contiguous():
        return True
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last):
        return True
    return False


class Segment:
    __slots__ = ("param", "offset", "numel", "group", "index")

    def __init__(self, param: torch.nn.Parameter, offset: int, numel: int, group: int,
                 index: int) -> None:
        self.param = param
        self.offset = offset
        self.numel = numel
        self.group = group
        self.index = index  # position in the optimizer's flattened param list


class FlatBuffer:
    """All parameters of one dtype: flat data + flat grad + the segment table."""

    def __init__(self, dtype: torch.dtype, device: torch.device) -> None:
        self.dtype = dtype
        self.device = device
        self.segments: List[Segment] = []
        self.numel = 0
        self.data: torch.Tensor = torch.empty(0)
        self.grad: torch.Tensor = torch.empty(0)
        # [start, end) of each optimizer param group inside this buffer
        self.group_ranges: Dict[int, Tuple[int, int]] = {}

    def view(self, flat: torch.Tensor, seg: Segment) -> torch.Tensor:
        p = seg.param
        return flat[seg.offset: seg.offset + seg.numel].as_strided(p.shape, p.stride())


class FlatParamSpace:
    """Flattens ``groups`` (list of param lists, one per optimizer param group)."""

    def __init__(self, groups: Sequence[Sequence[torch.nn.Parameter]], reverse: bool = True,
                 pad_multiple: int = 1) -> None:
        self.buffers: Dict[torch.dtype, FlatBuffer] = {}
        self.param_index: Dict[int, Tuple[torch.dtype, Segment]] = {}
        index = 0
        plan: Dict[torch.dtype, List[Tuple[int, int, torch.nn.Parameter]]] = {}
        for gi, params in enumerate(groups):
            for p in params:
                if not p.requires_grad:
                    index += 1
                    continue
                if id(p) in self.param_index or any(id(p) == id(q) for _, _, q in plan.get(p.dtype, [])):
                    raise ValueError("a parameter appears twice in the optimizer param groups")
                plan.setdefault(p.dtype, []).append((gi, index, p))
                index += 1
        for dtype, items in plan.items():
            device = items[0][2].device
            buf = FlatBuffer(dtype, device)
            # group-major, reverse registration order inside the group
            by_group: Dict[int, List[Tuple[int, torch.nn.Parameter]]] = {}
            for gi, idx, p in items:
                by_group.setdefault(gi, []).append((idx, p))
            off = 0
            for gi in sorted(by_group):
                members = by_group[gi][::-1] if reverse else by_group[gi]
                start = off
                for idx, p in members:
                    if p.device != device:
                        raise ValueError("all parameters of one dtype must live on one device")
                    seg = Segment(p, off, p.numel(), gi, idx)
                    buf.segments.append(seg)
                    self.param_index[id(p)] = (dtype, seg)
                    off += _round_up(p.numel(), ALIGN)
                buf.group_ranges[gi] = (start, off)
            # ZeRO partitions each buffer into world_size * ALIGN-element units: pad the tail.
            off = _round_up(off, max(1, pad_multiple))
            buf.numel = off
            buf.data = torch.zeros(off, dtype=dtype, device=device)
            buf.grad = torch.zeros(off, dtype=dtype, device=device)
            with torch.no_grad():
                for seg in buf.segments:
                    p = seg.param
                    if not _dense_strides(p):
                        p.data = p.data.contiguous()
                    v = buf.view(buf.data, seg)
                    v.copy_(p.data)
                    p.data = v
                    g = buf.view(buf.grad, seg)
                    if p.grad is not None:
                        g.copy_(p.grad)
                    p.grad = g
                    # fused kernels may accumulate straight into this persistent .grad view
                    # (see ops.batchnorm._direct_grad_targets)
                    p._dca_direct_grad = True
            self.buffers[dtype] = buf

    # ------------------------------------------------------------------ helpers
    def __iter__(self):
        return iter(self.buffers.values())

    def segment(self, p: torch.nn.Parameter) -> Optional[Segment]:
        hit = self.param_index.get(id(p))
        return hit[1] if hit else None

    def buffer_of(self, p: torch.nn.Parameter) -> Optional[FlatBuffer]:
        hit = self.param_index.get(id(p))
        return self.buffers[hit[0]] if hit else None

    def params(self) -> Iterable[torch.nn.Parameter]:
        for buf in self.buffers.values():
            for seg in buf.segments:
                yield seg.param

    def release_direct_grad(self) -> None:
        """Stop fused kernels from accumulating into these parameters' ``.grad`` (needed before
        driving backward with ``torch.autograd.grad`` over them; see ``ops._grad``)."""
        for p in self.params():
            p._dca_direct_grad = False

    def zero_grad(self) -> None:
        from determined_clone_amd.ops import _grad

        _grad.join()  # side-stream weight gradients may still be accumulating
        for buf in self.buffers.values():
            buf.grad.zero_()
        self.ensure_views()

    def ensure_views(self) -> None:
        """Re-install ``p.grad`` / ``p.data`` views if user code replaced them (e.g. a
        ``zero_grad(set_to_none=True)`` or ``p.data = ...``); copies any foreign grad in."""
        with torch.no_grad():
            for buf in self.buffers.values():
                base_d = buf.data.data_ptr()
                base_g = buf.grad.data_ptr()
                esz = buf.data.element_size()
                for seg in buf.segments:
                    p = seg.param
                    want_d = base_d + seg.offset * esz
                    if p.data.data_ptr() != want_d:
                        v = buf.view(buf.data, seg)
                        v.copy_(p.data)
                        p.data = v
                    g = p.grad
                    want_g = base_g + seg.offset * esz
                    if g is None:
                        buf.view(buf.grad, seg).zero_()
                        p.grad = buf.view(buf.grad, seg)
                    elif g.data_ptr() != want_g:
                        v = buf.view(buf.grad, seg)
                        v.copy_(g)
                        p.grad = v

    def grads_are_views(self) -> bool:
        for buf in self.buffers.values():
            base_g = buf.grad.data_ptr()
            esz = buf.grad.element_size()
            for seg in buf.segments:
                g = seg.param.grad
                if g is None or g.data_ptr() != base_g + seg.offset * esz:
                    return False
        return True
