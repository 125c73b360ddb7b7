"""NHWC convolutions for the ResNet / UNet hot path: the hand-written implicit-GEMM MFMA kernels of
``csrc/conv_igemm.hip`` (3x3 forward with the next BatchNorm's statistics in its epilogue, stride-1
data gradient -- optionally with the preceding BatchNorm's backward statistics in its epilogue --
and weight gradient) and, for 1x1 convolutions, a per-shape, per-direction choice between MIOpen,
hipBLASLt GEMMs on the NHWC row view and the implicit GEMM (decisions shipped in
``ops/tuned/conv_choices_gfx950.json``). Weight gradients accumulate straight into the parameters'
persistent ``.grad`` views when the optimizer's flat buffers own them (``ops/_grad.py``).
CPU / unsupported shapes: ``torch.nn.functional.conv2d`` (also the fp32 oracle of the GPU tests).

Fused statistics ride on the output tensor as ``y._dca_bn_partials`` and
``ops.batchnorm.batch_norm_act`` picks them up when it normalises exactly that tensor.

(An earlier hand-written pointwise GEMM family lost to the libraries on the forward / data
gradient by 1.3-2.4x at ResNet-50 shapes -- ``profiles/r8_pointwise_conv_study.txt`` -- and was
removed; the implicit GEMM covers 1x1 where it wins.)
"""
import os
import sys
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import _ext, _grad

# ----------------------------------------------------------------------------- library chooser
# Measured per direction on MI355X (tools/bench_conv_ops.py, profiles/s2_conv_ops_miopen_vs_gemm.txt):
# for a 1x1 convolution in NHWC the backward-data product dX[rows, Cin] = dY[rows, Cout] @ W is a
# plain GEMM, and hipBLASLt runs it 1.3-1.8x faster than MIOpen's implicit-GEMM solvers on most
# ResNet-50 shapes (MIOpen also zero-fills its output first); MIOpen stays ahead on the
# 64-channel layer1 shapes, on most forwards and on every weight gradient (a GEMM reducing over
# 10^5-10^6 rows, where hipBLASLt has no split-K tile). Which one runs is decided per shape and
# direction by timing both once, on the first training call (like cudnn.benchmark), and cached.
_CHOICE = {}
AUTOTUNE = os.environ.get("DCA_CONV_AUTOTUNE", "1") != "0"

# Shipped decisions (like the MIOpen find DB and the TunableOp CSV in ops/tuned/): every
# (direction, shape) this chooser met in the ResNet-50 bench (bs 1024, 256), the SD UNet bench and
# the CIFAR ASHA trials, timed on an MI355X by ``tools/dump_conv_choices.py`` and stored in
# ``ops/tuned/conv_choices_gfx950.json``. Shapes found there are never timed again: no timing
# noise between processes (16 ASHA trials on one GPU timing against each other's load) and
# identical decisions on every DDP rank. ``DCA_CONV_CHOICES=0`` ignores the file,
# ``DCA_CONV_CHOICES=<path>`` reads another one.
TIMINGS = 0  # candidates timed by this process (0 in a bench run whose shapes are all shipped)
_SHIPPED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "conv_choices_gfx950.json")


def _key_to_json(key) -> list:
    return [str(k) if isinstance(k, torch.dtype) else (list(k) if isinstance(k, tuple) else k) for k in key]


def _key_from_json(raw) -> tuple:
    out = []
    for k in raw:
        if isinstance(k, list):
            out.append(tuple(k))
        elif isinstance(k, str) and k.startswith("torch."):
            out.append(getattr(torch, k[len("torch."):]))
        else:
            out.append(k)
    return tuple(out)


def load_choices(path: Optional[str] = None) -> int:
    """Merge a decisions file into the cache (entries already decided in-process win)."""
    import json

    env = os.environ.get("DCA_CONV_CHOICES", "1")
    if path is None:
        if env == "0":
            return 0
        path = _SHIPPED_PATH if env == "1" else env
    if not os.path.exists(path):
        return 0
    with open(path) as f:
        data = json.load(f)
    n = 0
    for e in data.get("choices", []):
        key = _key_from_json(e["key"])
        if key not in _CHOICE:
            _CHOICE[key] = int(e["choice"])
            n += 1
    return n


def dump_choices(path: str, device_name: str = "") -> None:
    import json

    rows = [{"key": _key_to_json(k), "choice": v} for k, v in sorted(_CHOICE.items(), key=lambda kv: str(kv[0]))]
    with open(path, "w") as f:
        json.dump({"device": device_name, "choices": rows}, f, indent=1)


load_choices()

if os.environ.get("DCA_CONV_DUMP"):
    # record this process's decisions at exit (how the shipped file is produced: the bench
    # itself runs with DCA_CONV_CHOICES=0 DCA_CONV_DUMP=<path>, so every decision is timed under
    # the real step's conditions -- flat .grad views, side-stream weight gradients, allocator state)
    import atexit

    def _dump_at_exit() -> None:
        path = os.environ["DCA_CONV_DUMP"]
        merged = {}
        if os.path.exists(path):  # merge with decisions already in the file (other workloads)
            saved = dict(_CHOICE)
            _CHOICE.clear()
            load_choices(path)
            merged = dict(_CHOICE)
            _CHOICE.clear()
            _CHOICE.update(saved)
        merged.update(_CHOICE)
        _CHOICE.clear()
        _CHOICE.update(merged)
        dump_choices(path, torch.cuda.get_device_name(0) if torch.cuda.is_available() else "")

    atexit.register(_dump_at_exit)


def _time_us(fn, reps: int = 5) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def _world() -> int:
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


# Multi-rank runs: a shape missing from the shipped decisions takes candidate 0 (the library) on
# every rank without timing, so ranks cannot disagree and no collective is needed inside the
# forward (pipeline stages meet different shapes). DCA_CONV_AUTOTUNE_DIST=1 instead times on every
# rank and adopts rank 0's pick (broadcast_object_list; all ranks must meet the same shapes).
AUTOTUNE_DIST = os.environ.get("DCA_CONV_AUTOTUNE_DIST", "0") == "1"


def _choose(key, candidates) -> int:
    """Index of the fastest candidate for ``key`` (shipped, else timed once per process)."""
    got = _CHOICE.get(key)
    if got is not None:
        return got
    if not AUTOTUNE or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        return 0
    world = _world()
    if world > 1 and not AUTOTUNE_DIST:
        _CHOICE[key] = 0
        return 0
    global TIMINGS
    times = [_time_us(fn) for fn in candidates]
    TIMINGS += len(candidates)
    best = min(range(len(times)), key=times.__getitem__)
    if world > 1:
        import torch.distributed as dist

        obj = [best]
        dist.broadcast_object_list(obj, src=0)
        best = int(obj[0])
    _CHOICE[key] = best
    return best


def _rows(x: torch.Tensor, stride: int) -> torch.Tensor:
    """[N*Ho*Wo, C] matrix of an NHWC tensor (strided spatial subsample copied for stride > 1)."""
    v = x.permute(0, 2, 3, 1)
    if stride > 1:
        v = v[:, ::stride, ::stride, :]
    return v.reshape(-1, x.shape[1])


def _from_rows(m: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return m.view(n, h, w, m.shape[1]).permute(0, 3, 1, 2)  # channels_last NCHW view


# The backward-data GEMM of a 1x1 conv accumulates into its input's deposited identity-shortcut
# gradient (see _PointwiseLib; profiles/round3_shortcut_grad_accumulate_ab.txt), and a projection
# shortcut's data gradient is added at the strided positions by a HIP kernel (csrc/conv_igemm.hip
# strided_accumulate; ATen's strided add_ ran at 1.1-2.5 TB/s: round4_strided_accumulate_ab.txt).
ACC_HITS = 0  # backward passes that took the accumulate path (tests)


def _grad_sink(x: torch.Tensor):
    """The residual-gradient sink of a fused-BN output (ops/batchnorm.py ResidualGradSink), if any."""
    return getattr(x, "_dca_grad_sink", None)


def _pw_forward(x: torch.Tensor, weight: torch.Tensor, stride: int) -> torch.Tensor:
    n, cin, h, w = x.shape
    cout = weight.shape[0]
    ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    W = weight.view(cout, cin)

    def lib():
        return F.conv2d(x, weight, stride=stride)

    def gemm():
        return _from_rows(torch.mm(_rows(x, stride), W.t()), n, ho, wo)

    return (lib, gemm)[_choose(("fwd", tuple(x.shape), cout, stride, x.dtype), (lib, gemm))]()


# 1x1 forward on the implicit-GEMM MFMA kernel (csrc/conv_igemm.hip, R = S = 1) when its output
# feeds a training BatchNorm: the epilogue emits the BN's per-block statistics, so the BN skips its
# reduce pass over the output. Per shape, "auto" times {best library conv + BN forward} against
# {implicit GEMM with statistics + BN forward on them} once (like the other choosers) and keeps
# the faster; the backward stays on the library / GEMM paths below. DCA_IG1X1=1 forces, 0 disables.
IG1X1 = os.environ.get("DCA_IG1X1", "auto")


def _ig1x1_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if IG1X1 == "0" or not IGEMM or not x.is_cuda or torch.is_autocast_enabled():
        return False
    if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        return False
    n, cin, h, w = x.shape
    cout = weight.shape[0]
    if cin % 64 or cout % 64 or not weight.is_contiguous(memory_format=torch.channels_last):
        return False
    return x.numel() < 2 ** 30 and n * cout * h * w < 2 ** 30


def _ig1x1_wins(x: torch.Tensor, weight: torch.Tensor, stride: int) -> bool:
    if IG1X1 == "1":
        return True
    cout = weight.shape[0]
    key = ("fwd1x1+bn", tuple(x.shape), cout, stride, x.dtype)
    got = _CHOICE.get(key)
    if got is not None:  # decided: no timing tensors (4 small fills per call on the forward stream)
        return got == 1
    C = _ext.load()
    f = dict(device=x.device, dtype=torch.float32)
    g, b, rm, rv = torch.ones(cout, **f), torch.zeros(cout, **f), torch.zeros(cout, **f), torch.ones(cout, **f)

    def lib_then_bn():
        C.bn_fwd_train(_pw_forward(x, weight, stride), None, g, b, rm, rv, None, 0.1, 1e-5, True, None)

    def igemm_stats_then_bn():
        y, part = C.conv_igemm_fwd(x, weight, stride, 0, True)
        C.bn_fwd_train(y, None, g, b, rm, rv, None, 0.1, 1e-5, True, part)

    return _choose(key, (lib_then_bn, igemm_stats_then_bn)) == 1


class _PointwiseLib(torch.autograd.Function):
    """1x1 / no-padding convolution with per-direction library choice (MIOpen or hipBLASLt);
    with ``stats`` the forward runs on the implicit-GEMM kernel and also returns the following
    BatchNorm's partial statistics (an empty tensor otherwise)."""

    @staticmethod
    def forward(ctx, x, weight, stride, stats=False):
        if stats:
            y, partial = _ext.load().conv_igemm_fwd(x, weight, stride, 0, True)
        else:
            y, partial = _pw_forward(x, weight, stride), x.new_empty(0, dtype=torch.float32)
        ctx.mark_non_differentiable(partial)
        ctx.set_materialize_grads(False)  # autograd would zero-fill a gradient for `partial`
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        # x is a fused BN output whose identity-shortcut gradient arrives through a sink
        # (ops/batchnorm.py ResidualGradSink): the backward-data GEMM can accumulate into it
        ctx.sink = _grad_sink(x)
        return y, partial

    @staticmethod
    def backward(ctx, dy, _dpartial=None):
        x, weight = ctx.saved_tensors
        st = ctx.stride
        dy = dy.contiguous(memory_format=torch.channels_last)
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        args = (dy, x, weight, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1)
        bwd = torch.ops.aten.convolution_backward
        dx = dw = None
        if ctx.needs_input_grad[1]:  # issued first: on the side stream it overlaps the dgrad
            dw = _wgrad(args, weight)
        if ctx.needs_input_grad[0]:
            def lib():
                return bwd(*args, [True, False, False])[0]

            if st == 1:
                W = weight.view(cout, cin)

                def gemm():
                    return _from_rows(torch.mm(_rows(dy, 1), W), n, h, w)

                cands = (lib, gemm)
                pick = _choose(("dgrad", tuple(x.shape), cout, st, x.dtype), cands)
                acc = ctx.sink.grad if ctx.sink is not None else None
                rows = None
                if pick == 1 and acc is not None and acc.shape == x.shape and acc.dtype == dy.dtype \
                        and acc.is_contiguous(memory_format=torch.channels_last):
                    rows = _rows(acc, 1)
                    if rows.data_ptr() != acc.data_ptr():  # not a view: would accumulate into a copy
                        rows = None
                if rows is not None:
                    # dx = d(shortcut) + dy W as ONE GEMM with beta = 1 into the deposited
                    # shortcut gradient: the producing BN then reads one gradient tensor instead
                    # of two in both of its backward passes (one full-tensor pass saved per
                    # identity block)
                    rows.addmm_(_rows(dy, 1), W)
                    ctx.sink.grad = None
                    dx = acc
                    global ACC_HITS
                    ACC_HITS += 1
                else:
                    dx = cands[pick]()
            else:
                dx = lib()
        return dx, dw, None, None


class _PointwiseDual(torch.autograd.Function):
    """Two 1x1 convolutions of the SAME input -- a ResNet downsampling block's conv1 (stride 1)
    and its projection shortcut (stride s) -- with one input gradient: for s > 1 the shortcut's
    backward-data GEMM runs on the 1/s^2 subsampled rows only and is added in place into conv1's
    input gradient at the strided positions, instead of MIOpen writing a full-size, mostly-zero
    gradient (after zero-filling it) that autograd then sums with a full-size add."""

    @staticmethod
    def forward(ctx, x, w1, w2, stride, stats1=False, stats2=False):
        # statsN: that output runs on the implicit-GEMM kernel with its BN's partial statistics
        # (see _ig1x1_wins); an empty tensor stands in for partials not produced
        C = _ext.load()
        empty = x.new_empty(0, dtype=torch.float32)
        y1, p1 = C.conv_igemm_fwd(x, w1, 1, 0, True) if stats1 else (_pw_forward(x, w1, 1), empty)
        y2, p2 = C.conv_igemm_fwd(x, w2, stride, 0, True) if stats2 else (_pw_forward(x, w2, stride), empty)
        ctx.mark_non_differentiable(p1, p2)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for p1 / p2
        ctx.save_for_backward(x, w1, w2)
        ctx.stride = stride
        ctx.shapes = (y1.shape, y2.shape)
        return y1, y2, p1, p2

    @staticmethod
    def backward(ctx, dy1, dy2, _dp1=None, _dp2=None):
        x, w1, w2 = ctx.saved_tensors
        st = ctx.stride
        n, cin, h, w = x.shape
        bwd = torch.ops.aten.convolution_backward
        if dy1 is None or dy2 is None:  # one output unused (grads are not materialised)
            z = lambda s: x.new_zeros(s).contiguous(memory_format=torch.channels_last)  # noqa: E731
            dy1 = z(ctx.shapes[0]) if dy1 is None else dy1
            dy2 = z(ctx.shapes[1]) if dy2 is None else dy2
        dy1 = dy1.contiguous(memory_format=torch.channels_last)
        dy2 = dy2.contiguous(memory_format=torch.channels_last)
        a1 = (dy1, x, w1, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        a2 = (dy2, x, w2, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1)
        dx = None
        dw1 = _wgrad(a1, w1) if ctx.needs_input_grad[1] else None
        dw2 = _wgrad(a2, w2) if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[0]:
            W1 = w1.view(w1.shape[0], cin)
            c1 = (lambda: bwd(*a1, [True, False, False])[0],
                  lambda: _from_rows(torch.mm(_rows(dy1, 1), W1), n, h, w))
            dx = c1[_choose(("dgrad", tuple(x.shape), w1.shape[0], 1, x.dtype), c1)]()
            W2 = w2.view(w2.shape[0], cin)
            if st == 1:
                c2 = (lambda: bwd(*a2, [True, False, False])[0],
                      lambda: _from_rows(torch.mm(_rows(dy2, 1), W2), n, h, w))
                pick = _choose(("dgrad", tuple(x.shape), w2.shape[0], 1, x.dtype), c2)
                rows = _rows(dx, 1) if pick == 1 and \
                    dx.is_contiguous(memory_format=torch.channels_last) else None
                if rows is not None and rows.data_ptr() == dx.data_ptr():
                    rows.addmm_(_rows(dy2, 1), W2)  # beta = 1: no separate full-size add
                else:
                    dx.add_(c2[pick]())
            else:
                ho, wo = dy2.shape[2], dy2.shape[3]
                small = torch.mm(_rows(dy2, 1), W2).view(n, ho, wo, cin)
                if dx.dtype == torch.bfloat16 and cin % 8 == 0 and \
                        dx.is_contiguous(memory_format=torch.channels_last):
                    # HIP kernel: 16-B lanes at HBM rate (ATen's strided add ran at 1.1-2.5 TB/s)
                    _ext.load().strided_accumulate(dx, small.permute(0, 3, 1, 2), st)
                else:
                    dx.permute(0, 2, 3, 1)[:, ::st, ::st, :].add_(small)
        return dx, dw1, dw2, None, None, None


def pointwise_dual(conv1: nn.Conv2d, proj: nn.Conv2d, x: torch.Tensor, bn_stats: bool = False):
    """``(conv1(x), proj(x))`` for a downsampling bottleneck (see :class:`_PointwiseDual`); with
    ``bn_stats`` each output may carry its BatchNorm's partial statistics (``_ig1x1_wins``)."""
    if (_lib_supported(conv1, x) and _lib_supported(proj, x)
            and conv1.stride == (1, 1)):
        x = x.contiguous(memory_format=torch.channels_last)
        s1 = bool(bn_stats) and _ig1x1_ok(x, conv1.weight) and _ig1x1_wins(x, conv1.weight, 1)
        s2 = bool(bn_stats) and _ig1x1_ok(x, proj.weight) and _ig1x1_wins(x, proj.weight, proj.stride[0])
        y1, y2, p1, p2 = _PointwiseDual.apply(x, conv1.weight, proj.weight, proj.stride[0], s1, s2)
        if s1:
            y1._dca_bn_partials = p1
        if s2:
            y2._dca_bn_partials = p2
        return y1, y2
    return pointwise_conv(conv1, x, bn_stats), pointwise_conv(proj, x, bn_stats)


# Weight gradients: MIOpen's backward-weight solvers or the split-pixel implicit-GEMM MFMA kernel
# of csrc/conv_igemm.hip (numerics: tools/bench_igemm.py, tests/test_conv_gpu.py). "auto" times
# both once per shape (like cudnn.benchmark) and keeps the faster; "1" / "0" force one.
IGEMM_WGRAD = os.environ.get("DCA_IGEMM_WGRAD", "auto")


def _igemm_wgrad_ok(args) -> bool:
    dy, x, w = args[0], args[1], args[2]
    stride, pad, dil, groups = args[4], args[5], args[6], args[9]
    if IGEMM_WGRAD == "0" or not IGEMM or not x.is_cuda or args[7]:  # transposed conv
        return False
    if x.dtype != torch.bfloat16 or dy.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if groups != 1 or list(dil) != [1, 1] or stride[0] != stride[1] or pad[0] != pad[1]:
        return False
    if w.shape[2] != w.shape[3] or pad[0] >= w.shape[2] or x.shape[1] % 64 or w.shape[0] % 64:
        return False
    if not (x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last)):
        return False
    m = dy.shape[0] * dy.shape[2] * dy.shape[3]
    return m < 2 ** 24 and x.numel() < 2 ** 30 and dy.numel() < 2 ** 30


def _wgrad(args, weight: torch.Tensor) -> Optional[torch.Tensor]:
    """Weight gradient of ``convolution_backward(*args)``: on the side stream (accumulated into
    ``weight.grad``, returns None) when the parameter has a persistent ``.grad`` view
    (``ops/_grad.py``; ``DCA_WGRAD_STREAM=0`` disables), else computed inline and returned."""
    bwd = torch.ops.aten.convolution_backward
    dy, x = args[0], args[1]
    use_ours = False
    if _igemm_wgrad_ok(args):
        st, pad = args[4][0], args[5][0]
        if IGEMM_WGRAD == "1":
            use_ours = True
        else:
            cands = (lambda: bwd(*args, [False, True, False])[1],
                     lambda: _ext.load().conv_igemm_wgrad(dy, x, args[2], st, pad))
            use_ours = _choose(("wgrad", tuple(x.shape), tuple(args[2].shape), st, pad), cands) == 1

    def compute(acc=None):
        if use_ours:
            return _ext.load().conv_igemm_wgrad(dy, x, args[2], args[4][0], args[5][0], acc)
        dw = bwd(*args, [False, True, False])[1]
        return acc.add_(dw) if acc is not None else dw

    s = _grad.side_stream_for(weight)
    if s is None:
        return compute()
    _grad.fork(s, (dy, x))
    with torch.cuda.stream(s):
        compute(_grad.target(weight))
    return None


class _SpatialConv(torch.autograd.Function):
    """k x k convolution (groups 1, optional bias) whose backward issues the weight (and bias)
    gradient on the side stream before the data gradient (``ops/_grad.py``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding):
        ctx.save_for_backward(x, weight)
        ctx.stride, ctx.padding = stride, padding
        ctx.bias = bias
        return F.conv2d(x, weight, bias, stride, padding)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        args = (dy, x, w, None, list(ctx.stride), list(ctx.padding), [1, 1], False, [0, 0], 1)
        dw = _wgrad(args, w) if ctx.needs_input_grad[1] else None
        db = _bgrad(dy, ctx.bias) if ctx.bias is not None and ctx.needs_input_grad[2] else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        return dx, dw, db, None, None


def _bgrad(dy: torch.Tensor, bias: torch.Tensor) -> Optional[torch.Tensor]:
    """Bias gradient (sum of dy over N, H, W): on the side stream into ``bias.grad`` when it is a
    persistent view, else returned to autograd."""
    s = _grad.side_stream_for(bias)
    if s is None:
        return dy.sum((0, 2, 3), dtype=torch.float32).to(bias.dtype)
    _grad.fork(s, (dy,))
    with torch.cuda.stream(s):
        _grad.target(bias).add_(dy.sum((0, 2, 3), dtype=torch.float32).to(bias.dtype))
    return None


# ----------------------------------------------------------------------------- ResNet stem
# The 7x7 / stride-2 stem on a 3-channel image is MIOpen's least efficient convolution of the model
# (140 TFLOP/s forward, 175 weight gradient at bs 1024: 3-channel pixels are 6-byte rows). Rewritten
# by space-to-depth -- pad the image by 3, fold each 2x2 pixel block into 12 channels, pad the
# kernel to 8x8 and fold it the same way -- it is exactly a 4x4 / stride-1 convolution on a
# 115x115x12 image: 1119 us forward + 934 us weight gradient instead of 1716 + 1381
# (profiles/round3_stem_conv_variants_find.txt); +0.5% end to end with its find-DB entries shipped
# (profiles/round3_stem_s2d_ab.txt).


# the stem image's pad + space-to-depth runs as one HIP pass (csrc/conv_igemm.hip stem_s2d_kernel).
# (Measured and removed in round 6: an MFMA stem convolution kernel with the BatchNorm statistics in
# its epilogue, a hand-written stem weight gradient and a 16-channel S2D tensor on MIOpen -- each
# lost in the step: profiles/round5_stem_conv_kernel_ab.txt, round5_stem_wgrad_kernel_ab.txt.)


def _s2d_input(x: torch.Tensor) -> torch.Tensor:
    """[N, 3, H, W] (NHWC memory) -> [N, 12, (H+6)/2, (W+6)/2] channels_last, channel (dy, dx, c)."""
    n, c, h, w = x.shape
    if x.is_cuda and x.dtype == torch.bfloat16 and c == 3:
        return _ext.load().stem_s2d(x)  # one pass, padding folded in (csrc/conv_igemm.hip)
    xn = F.pad(x.permute(0, 2, 3, 1), (0, 0, 3, 3, 3, 3))  # [N, H+6, W+6, C]
    hh, ww = (h + 6) // 2, (w + 6) // 2
    xs = xn.view(n, hh, 2, ww, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(n, hh, ww, 4 * c)
    return xs.permute(0, 3, 1, 2)


def _s2d_weight(w: torch.Tensor) -> torch.Tensor:
    """[K, C, 7, 7] -> [K, 4C, 4, 4] (channels_last), channel (dy, dx, c), tap (i, j) = (2i+dy, 2j+dx)."""
    k, c = w.shape[:2]
    wp = F.pad(w, (0, 1, 0, 1)).view(k, c, 4, 2, 4, 2).permute(0, 3, 5, 1, 2, 4).reshape(k, 4 * c, 4, 4)
    return wp.contiguous(memory_format=torch.channels_last)


def _s2d_weight_grad(dw2: torch.Tensor, c: int) -> torch.Tensor:
    """Inverse of :func:`_s2d_weight` for the gradient: [K, 4C, 4, 4] -> [K, C, 7, 7]."""
    k = dw2.shape[0]
    d = dw2.reshape(k, 2, 2, c, 4, 4).permute(0, 3, 4, 1, 5, 2).reshape(k, c, 8, 8)
    return d[:, :, :7, :7]


class _StemS2D(torch.autograd.Function):
    """7x7/2 (padding 3) convolution of a 3-channel image as the space-to-depth 4x4/1 convolution
    (MIOpen on the 12-channel form). The weight gradient is folded back to 7x7 and, on a GPU, runs on
    the side stream into the parameter's ``.grad`` view (``ops/_grad.py``). The image gets no
    gradient."""

    @staticmethod
    def forward(ctx, x, weight):
        ctx.set_materialize_grads(False)
        xs = _s2d_input(x)
        w2 = _s2d_weight(weight)
        ctx.save_for_backward(xs, w2)
        ctx.weight = weight
        return F.conv2d(xs, w2)

    @staticmethod
    def backward(ctx, dy):
        xs, w2 = ctx.saved_tensors
        weight = ctx.weight
        if dy is None:
            return None, None
        dy = dy.contiguous(memory_format=torch.channels_last)
        c = weight.shape[1]

        def wgrad():
            args = (dy, xs, w2, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
            return torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        s = _grad.side_stream_for(weight)
        if s is None:
            return None, _s2d_weight_grad(wgrad(), c).to(weight.dtype)
        _grad.fork(s, (dy, xs))
        with torch.cuda.stream(s):
            _grad.target(weight).add_(_s2d_weight_grad(wgrad(), c))
        return None, None


def stem_conv(conv: nn.Conv2d, x: torch.Tensor, bn_stats: bool = False) -> torch.Tensor:
    """The ResNet stem convolution: space-to-depth form on a GPU when it applies (7x7, stride 2,
    padding 3, 3 input channels, no bias, even H and W, image without gradient), else
    :func:`spatial_conv`. The S2D form is pinned to the 7x7 path only for zero padding, matching
    input / weight dtypes and no autocast (its saved tensors keep their own dtype). ``bn_stats`` is
    accepted for call-site symmetry (the stem output carries no fused statistics)."""
    if (x.is_cuda and not x.requires_grad and conv.kernel_size == (7, 7)
            and conv.padding_mode == "zeros" and x.dtype == conv.weight.dtype
            and not torch.is_autocast_enabled()
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.in_channels == 3
            and conv.groups == 1 and conv.bias is None and conv.dilation == (1, 1)
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0):
        return _StemS2D.apply(x.contiguous(memory_format=torch.channels_last), conv.weight)
    return spatial_conv(conv, x)


# ----------------------------------------------------------------------------- k x k implicit GEMM
# ResNet-50's 3x3 convolutions on the hand-written MFMA implicit-GEMM kernel (csrc/conv_igemm.hip):
# the forward also emits the following BatchNorm's per-block statistics (its reduce pass over HBM
# is skipped), the stride-1 data gradient runs on the same kernel (flipped, transposed weight).
# Measured at bs 1024 against MIOpen (tools/bench_igemm.py, profiles/round4_igemm_v2_stages.txt):
# forward at parity (5.23 vs 5.18 ms per step, before counting the statistics pass it removes),
# stride-1 data gradient 4.16 vs 5.56 ms. Stride-2 data gradients and every weight gradient stay
# on MIOpen (the latter on the side stream). DCA_IGEMM=0 routes everything back to MIOpen.
IGEMM = os.environ.get("DCA_IGEMM", "1") != "0"


def igemm_supported(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (IGEMM and x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16):
        return False
    w = conv.weight
    k = conv.kernel_size
    if k[0] != k[1] or k[0] < 2 or conv.stride[0] != conv.stride[1] or conv.groups != 1:
        return False
    if conv.dilation != (1, 1) or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    if not isinstance(conv.padding, tuple) or conv.padding[0] != conv.padding[1] or conv.padding[0] >= k[0]:
        return False
    if conv.in_channels % 64 or conv.out_channels % 64 or w.dtype != torch.bfloat16:
        return False
    if not w.is_contiguous(memory_format=torch.channels_last) or torch.is_autocast_enabled():
        return False
    n, c, h, ww = x.shape
    return n * c * h * ww < 2 ** 30 and n * conv.out_channels * h * ww < 2 ** 30


class _IgemmConv(torch.autograd.Function):
    """k x k convolution on conv_igemm.hip; returns ``(y, bn_partials)``."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, stats):
        y, partial = _ext.load().conv_igemm_fwd(x, weight, stride, pad, stats)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.save_for_backward(x, weight)
        ctx.stride, ctx.pad = stride, pad
        if partial is not None:
            ctx.mark_non_differentiable(partial)
        return y, partial

    @staticmethod
    def backward(ctx, dy, _dpartial):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        st, pad = ctx.stride, ctx.pad
        args = (dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1)
        dw = _wgrad(args, w) if ctx.needs_input_grad[1] else None
        dx = None
        if ctx.needs_input_grad[0]:
            if st == 1:
                dx = _ext.load().conv_igemm_dgrad(dy, w, pad)
            else:
                dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        return dx, dw, None, None, None


def spatial_conv(conv: nn.Conv2d, x: torch.Tensor, bn_stats: bool = False) -> torch.Tensor:
    """``conv(x)``; on a GPU, k x k bf16 convolutions run on the implicit-GEMM kernel (with
    ``bn_stats`` the output carries the following BatchNorm's partial statistics), others on
    MIOpen with the weight (and bias) gradient on the side stream (``ops/_grad.py``)."""
    if igemm_supported(conv, x):
        x = x.contiguous(memory_format=torch.channels_last)
        y, partial = _IgemmConv.apply(x, conv.weight, conv.stride[0], conv.padding[0], bool(bn_stats))
        if partial is not None:
            y._dca_bn_partials = partial
        return y
    if (_grad.SIDE_STREAM and x.is_cuda and conv.groups == 1 and conv.dilation == (1, 1)
            and isinstance(conv.padding, tuple) and conv.training and conv.weight.requires_grad
            and conv.padding_mode == "zeros"):
        return _SpatialConv.apply(x.contiguous(memory_format=torch.channels_last), conv.weight,
                                  conv.bias, conv.stride, conv.padding)
    return nn.Conv2d.forward(conv, x)  # (not conv(x): subclasses route their forward here)


def _lib_supported(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float16)):
        return False
    if conv.kernel_size != (1, 1) or conv.padding != (0, 0) or conv.stride[0] != conv.stride[1]:
        return False
    if conv.groups != 1 or conv.dilation != (1, 1) or conv.bias is not None:
        return False
    w = conv.weight
    return w.dtype == x.dtype and w.is_contiguous(memory_format=torch.channels_last)


def pointwise_conv(conv: nn.Conv2d, x: torch.Tensor, bn_stats: bool = False) -> torch.Tensor:
    """``conv(x)`` for a 1x1 convolution in NHWC: each direction runs on the fastest of MIOpen,
    hipBLASLt and the implicit GEMM for its shape; with ``bn_stats`` and the implicit-GEMM forward
    the output carries the next BatchNorm's partial statistics from its epilogue."""
    if _lib_supported(conv, x):
        x = x.contiguous(memory_format=torch.channels_last)
        stats = bool(bn_stats) and _ig1x1_ok(x, conv.weight) and _ig1x1_wins(x, conv.weight, conv.stride[0])
        y, partial = _PointwiseLib.apply(x, conv.weight, conv.stride[0], stats)
        if stats:
            y._dca_bn_partials = partial
        return y
    return conv(x)


def take_bn_partials(x: torch.Tensor) -> Optional[torch.Tensor]:
    """The fused statistics attached to ``x`` by :func:`pointwise_conv` (consumed once)."""
    p = getattr(x, "_dca_bn_partials", None)
    if p is not None:
        x._dca_bn_partials = None
    return p
