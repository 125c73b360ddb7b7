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
    if g is None or g.dtype != p.dtype or g.shape != p.shape:
        return None
    # dense in the parameter's own layout: contiguous, or a channels_last convolution weight
    # (FlatParamSpace gives .grad the parameter's strides; the k x k weight-gradient paths --
    # MIOpen + add_, the implicit-GEMM kernel's KRSC store, the stem's add_ -- all take either.
    # Requiring plain contiguity kept every 3x3 / 7x7 weight gradient of a channels_last ResNet
    # off the side stream: 17 MIOpen backward-weight calls, ~6.5 ms of a 80 ms step, on the
    # critical path -- profiles/round4_resnet50_step_breakdown_default.txt)
    if not (g.is_contiguous() or (g.dim() == 4 and g.stride() == p.stride()
                                  and g.is_contiguous(memory_format=torch.channels_last))):
        return None
    if g.dtype not in (torch.float32, torch.bfloat16):
        return None
    return g


# ----------------------------------------------------------------------------- side stream
# Weight gradients (a convolution's backward-weight, reducing over every output position) are
# off the backward critical path: nothing downstream of them runs until the optimizer step. They
# run on a second HIP stream (``DCA_WGRAD_STREAM=0`` turns this off), accumulated straight into the
# parameter's persistent ``.grad`` view, so the compute-bound MFMA weight-gradient kernels overlap
# the bandwidth-bound BatchNorm / data-gradient kernels of the layers before them. Everything that
# reads gradients joins the side stream first: the bucketed all-reduce launches its collective on
# the side stream (after an event from the main stream), and ``join()`` -- called at the end of
# ``context.backward``, before any fused optimizer step / grad-norm and before ``zero_grad`` --
# makes the current stream wait for it. Measured on ResNet-50 bs256 (1x MI355X, same-box A/B,
# profiles/round2_wgrad_side_stream_ab.txt): 9754 -> 10043 img/s.
SIDE_STREAM = os.environ.get("DCA_WGRAD_STREAM", "1") != "0"
_streams = {}
_pending = set()
# Tensors the side stream reads are kept alive by reference until join() instead of
# ``record_stream``: with record_stream every activation / gradient block freed during backward
# stays unusable until the lagging side stream passes it, the next forward cannot reuse it, and
# the caching allocator grew a ResNet-50 bs-1024 process to 222 GB reserved for 42.5 GB of live
# tensors -- past the HBM left on a box where another process still held memory, where every
# allocation miss became a 1-25 s free-all-and-retry (profiles/round4_bench_slow_mode.txt).
# Released after the current stream has waited for the side stream, the blocks return to the
# current stream's pool immediately reusable. Entries whose side-stream reads have demonstrably
# finished (an event recorded after them has completed) are dropped earlier, at the next fork, so
# code that runs several backward passes before an optimizer step (and so before join()) holds
# only what the side stream has not reached yet. DCA_WGRAD_KEEPALIVE=0 restores record_stream.
KEEPALIVE = os.environ.get("DCA_WGRAD_KEEPALIVE", "1") != "0"
_keep = []  # [tensors, event recorded on the side stream after their readers (or None yet)]


def side_stream_for(p: Optional[torch.Tensor]) -> Optional["torch.cuda.Stream"]:
    """The side stream to run ``p``'s weight gradient on, or None (feature off, CPU, graph
    capture, or no persistent ``.grad`` to accumulate into)."""
    if not SIDE_STREAM or p is None or not p.is_cuda or target(p) is None:
        return None
    if torch.cuda.is_current_stream_capturing():
        return None
    dev = p.device.index
    s = _streams.get(dev)
    if s is None:
        s = _streams[dev] = torch.cuda.Stream(device=p.device)
    return s


def fork(stream: "torch.cuda.Stream", tensors=()) -> None:
    """Order ``stream`` after the work queued so far on the current stream; keep ``tensors``
    (allocated on the current stream) alive until ``stream`` has used them."""
    if KEEPALIVE and _keep and _keep[-1][1] is None:
        # everything the previous fork's caller queued on the side stream precedes this event
        done = torch.cuda.Event()
        done.record(stream)
        _keep[-1][1] = done
    while KEEPALIVE and _keep and _keep[0][1] is not None and _keep[0][1].query():
        _keep.pop(0)  # those reads have executed: the blocks may be reused by the current stream
    ev = torch.cuda.Event()
    ev.record()
    stream.wait_event(ev)
    live = [t for t in tensors if t is not None]
    if KEEPALIVE:
        if live:
            _keep.append([live, None])
    else:
        for t in live:
            t.record_stream(stream)
    _pending.add(stream)


def pending() -> bool:
    return bool(_pending)


def join() -> None:
    """Make the current stream wait for all side-stream gradient work."""
    if not _pending:
        return
    cur = torch.cuda.current_stream()
    for s in list(_pending):
        cur.wait_stream(s)
    _pending.clear()
    _keep.clear()  # the current stream is now ordered after every side-stream read


def comm_stream() -> Optional["torch.cuda.Stream"]:
    """Stream a gradient collective should be issued on when side-stream gradients are in flight
    (ordered after the main stream's work so far), else None."""
    if not _pending:
        return None
    s = next(iter(_pending))
    fork(s)
    return s


# ----------------------------------------------------------------------------- step stream
# The training step's critical path (forward, data gradients, optimizer) runs on the current
# stream while the weight gradients queue on the side stream: when both have work ready the
# hardware dispatches their workgroups in queue-priority order. With DCA_STEP_STREAM_PRIORITY=high
# the controllers run the step on a high-priority stream, so side-stream work fills the CUs the
# critical path leaves idle instead of delaying it.
import contextlib  # noqa: E402

STEP_PRIORITY = os.environ.get("DCA_STEP_STREAM_PRIORITY", "normal")


@contextlib.contextmanager
def step_stream(device: Optional[torch.device] = None):
    """Run the enclosed training loop on a high-priority stream (``DCA_STEP_STREAM_PRIORITY=high``
    on a GPU), ordered after the work queued so far and joined back at the end."""
    if STEP_PRIORITY != "high" or not torch.cuda.is_available() or \
            (device is not None and device.type != "cuda"):
        yield None
        return
    _, greatest = torch.cuda.Stream.priority_range()
    prev = torch.cuda.current_stream()
    s = torch.cuda.Stream(priority=greatest)
    s.wait_stream(prev)
    with torch.cuda.stream(s):
        try:
            yield s
        finally:
            join()
    prev.wait_stream(s)
