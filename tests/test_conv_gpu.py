"""Numerics of the convolution paths (ops/conv.py: library 1x1 choices, implicit-GEMM MFMA kernels of
ops/csrc/conv_igemm.hip, fused BatchNorm statistics) vs fp32 PyTorch."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from determined_clone_amd.ops import _ext, batchnorm, conv

pytestmark = pytest.mark.gpu

def _close(got, ref, tol, what):
    err = (got.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol * scale, f"{what}: max abs err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("choice", [0, 1])
@pytest.mark.parametrize("shape,stride", [((4, 256, 28, 28, 128), 1), ((2, 64, 15, 17, 256), 1),
                                          ((4, 256, 28, 28, 512), 2), ((3, 1024, 14, 14, 256), 1)])
def test_pointwise_library_choice_matches_fp32(shape, stride, choice):
    """Both library paths of ops.conv._PointwiseLib (MIOpen / hipBLASLt GEMM on the NHWC row
    view), forced per direction, against an fp32 F.conv2d reference."""
    N, ci, H, W, co = shape
    torch.manual_seed(0)
    c = nn.Conv2d(ci, co, 1, stride=stride, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(N, ci, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    conv._CHOICE.clear()
    for d in ("fwd", "dgrad"):
        conv._CHOICE[(d, tuple(x.shape), co, stride, x.dtype)] = choice
    try:
        x1 = x.clone().requires_grad_(True)
        y = conv.pointwise_conv(c, x1)
        assert y.is_contiguous(memory_format=torch.channels_last)
        g = torch.randn_like(y)
        y.backward(g)
        x2 = x.float().clone().requires_grad_(True)
        w2 = c.weight.detach().float().clone().requires_grad_(True)
        y2 = F.conv2d(x2, w2, stride=stride)
        y2.backward(g.float())
        _close(y, y2, 2e-2, "fwd")
        _close(x1.grad, x2.grad, 2e-2, "dgrad")
        _close(c.weight.grad, w2.grad, 2e-2, "wgrad")
    finally:
        conv._CHOICE.clear()
        conv.load_choices()  # back to the shipped decisions for later tests


@pytest.mark.parametrize("dgrad_choice", [None, 0, 1])
@pytest.mark.parametrize("stride", [1, 2])
def test_pointwise_dual_matches_two_convs(stride, dgrad_choice):
    """conv1(x) and the projection shortcut proj(x) through ops.conv.pointwise_dual (one input
    gradient, the strided shortcut's dgrad accumulated in place -- for stride 1 on the GEMM path
    as one beta = 1 GEMM into conv1's gradient) against fp32 autograd; backward-data library
    chosen by the chooser, or forced to MIOpen (0) / the GEMM (1)."""
    torch.manual_seed(0)
    N, ci, H = 4, 256, 28
    c1 = nn.Conv2d(ci, 128, 1, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    cp = nn.Conv2d(ci, 512, 1, stride=stride, bias=False).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(N, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    conv._CHOICE.clear()
    if dgrad_choice is not None:
        for co in (128, 512):
            conv._CHOICE[("dgrad", tuple(x.shape), co, 1, x.dtype)] = dgrad_choice
    try:
        y1, yp = conv.pointwise_dual(c1, cp, x1)
        g1, gp = torch.randn_like(y1), torch.randn_like(yp)
        torch.autograd.backward([y1, yp], [g1, gp])
    finally:
        conv._CHOICE.clear()
        conv.load_choices()  # back to the shipped decisions for later tests
    x2 = x.float().clone().requires_grad_(True)
    w1 = c1.weight.detach().float().clone().requires_grad_(True)
    wp = cp.weight.detach().float().clone().requires_grad_(True)
    r1, rp = F.conv2d(x2, w1), F.conv2d(x2, wp, stride=stride)
    torch.autograd.backward([r1, rp], [g1.float(), gp.float()])
    _close(y1, r1, 2e-2, "y1")
    _close(yp, rp, 2e-2, "yp")
    _close(x1.grad, x2.grad, 2e-2, "dx")
    _close(c1.weight.grad, w1.grad, 2e-2, "dw1")
    _close(cp.weight.grad, wp.grad, 2e-2, "dwp")


@pytest.mark.parametrize("model_fn", ["tiny"])
def test_side_stream_weight_gradients_match_inline(monkeypatch, model_fn):
    """DCA_WGRAD_STREAM: conv weight gradients on the side stream, accumulated into the flat
    .grad views, match the inline path (same MIOpen solvers, same bf16 accumulation)."""
    from determined_clone_amd.models import resnet
    from determined_clone_amd.ops import _grad
    from determined_clone_amd.ops import optim as fopt

    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10)).to(dev)
    opt = fopt.FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=dev)
    grads = []
    # warm-up pass first: the convolution choosers (ops/conv.py _choose) time their candidates on
    # first use; the compared passes then run the same kernels. Inline twice gives the noise floor.
    for side in (False, False, False, True):
        monkeypatch.setattr(_grad, "SIDE_STREAM", side)
        opt.zero_grad()
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        if side:
            assert _grad.pending()
        _grad.join()
        torch.cuda.synchronize()
        grads.append([p.grad.float().clone() for p in model.parameters()])
    names = [n for n, _ in model.named_parameters()]
    for name, a, a2, b in zip(names, grads[1], grads[2], grads[3]):
        # MIOpen's split-K weight-gradient solvers reduce with atomics: compare in norm, above the
        # inline-vs-inline noise (bias gradients are sums with heavy cancellation)
        err, floor = (a - b).norm().item(), (a - a2).norm().item()
        assert err <= 2e-2 * a.norm().item() + 4 * floor + 1e-6, (name, err, floor, a.norm().item())
    # the optimizer step joins by itself when the caller did not
    monkeypatch.setattr(_grad, "SIDE_STREAM", True)
    opt.zero_grad()
    F.cross_entropy(model(x).float(), y).backward()
    opt.step()
    assert not _grad.pending()


def test_pointwise_igemm_with_bn_stats_matches_library_path(monkeypatch):
    """1x1 convolutions forced onto the implicit-GEMM kernel with the BatchNorm statistics in its
    epilogue (DCA_IG1X1=1) train the tiny bottleneck ResNet like the library path (IG1X1=0):
    same loss and gradients within bf16 noise, and the BNs really consumed fused statistics."""
    from determined_clone_amd.models import resnet
    from determined_clone_amd.ops import conv as conv_ops

    torch.manual_seed(0)
    dev = torch.device("cuda")
    base = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10)).to(dev)
    x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=dev)
    out = {}
    orig = conv_ops._PointwiseLib.apply
    for mode in ("0", "1"):
        monkeypatch.setattr(conv_ops, "IG1X1", mode)
        model = copy.deepcopy(base)
        hits = []

        def spy(*a, hits=hits):
            r = orig(*a)
            hits.append(bool(a[3]) if len(a) > 3 else False)
            return r

        monkeypatch.setattr(conv_ops._PointwiseLib, "apply", spy)
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        out[mode] = (loss.item(), [p.grad.float().clone() for p in model.parameters()])
        if mode == "1":
            assert sum(hits) >= 4, hits  # conv1 / conv3 of the blocks took the fused-stats path
    assert abs(out["0"][0] - out["1"][0]) < 2e-2 * max(1.0, abs(out["0"][0]))
    for a, b in zip(out["0"][1], out["1"][1]):
        assert (a - b).norm().item() <= 5e-2 * a.norm().item() + 1e-4


def test_side_stream_inputs_released_without_optimizer_step(monkeypatch):
    """Side-stream weight-gradient inputs are held by reference (not record_stream) until join();
    with several backward passes before any optimizer step (gradient accumulation in user code),
    the inputs whose side-stream reads have executed are dropped at the next fork, so the held set
    does not grow with the number of backward passes."""
    from determined_clone_amd.models import resnet
    from determined_clone_amd.ops import _grad
    from determined_clone_amd.ops import optim as fopt

    monkeypatch.setattr(_grad, "SIDE_STREAM", True)
    monkeypatch.setattr(_grad, "KEEPALIVE", True)
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = resnet.to_mi355x_layout(resnet.resnet18_bottleneck_tiny(num_classes=10)).to(dev)
    opt = fopt.FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=dev)
    opt.zero_grad()
    F.cross_entropy(model(x).float(), y).backward()
    per_pass = len(_grad._keep)
    assert per_pass > 0 and _grad.pending()
    for _ in range(3):
        torch.cuda.synchronize()  # the side stream has executed everything queued so far
        F.cross_entropy(model(x).float(), y).backward()
        assert len(_grad._keep) <= per_pass + 1, (len(_grad._keep), per_pass)
    opt.step()  # joins
    assert not _grad.pending() and not _grad._keep


@pytest.mark.parametrize("hw", [(224, 224), (64, 48), (2, 8), (6, 10)])
def test_stem_s2d_kernel_matches_pad_and_reshape(hw):
    """The HIP space-to-depth (padding folded in) is a pure data movement: bit-equal to the ATen
    pad + permute + reshape it replaces, including images smaller than the padding."""
    from determined_clone_amd.ops import _ext

    torch.manual_seed(0)
    x = torch.randn(3, 3, *hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xs = _ext.load().stem_s2d(x)
    n, c, h, w = x.shape
    ref = F.pad(x.permute(0, 2, 3, 1), (0, 0, 3, 3, 3, 3)).view(n, (h + 6) // 2, 2, (w + 6) // 2, 2, c)
    ref = ref.permute(0, 1, 3, 2, 4, 5).reshape(n, (h + 6) // 2, (w + 6) // 2, 4 * c).permute(0, 3, 1, 2)
    assert xs.is_contiguous(memory_format=torch.channels_last) and xs.shape == ref.shape
    assert torch.equal(xs, ref)


@pytest.mark.parametrize("side", [True, False])
@pytest.mark.parametrize("hw", [(224, 224), (64, 48)])
def test_stem_space_to_depth_matches_fp32(monkeypatch, side, hw):
    """The space-to-depth stem (7x7/2 as a 4x4/1 conv on 12 channels) equals the fp32 7x7
    convolution forward and weight gradient, inline and on the side stream."""
    from determined_clone_amd.ops import _grad
    from determined_clone_amd.parallel.flat import FlatParamSpace

    monkeypatch.setattr(_grad, "SIDE_STREAM", side)
    torch.manual_seed(0)
    c = nn.Conv2d(3, 64, 7, 2, 3, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    FlatParamSpace([[c.weight]])  # persistent .grad view (side-stream accumulation target)
    x = torch.randn(4, 3, *hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = conv.stem_conv(c, x)
    ref = F.conv2d(x.float(), c.weight.float(), stride=2, padding=3)
    _close(y, ref, 2e-2, "stem fwd")
    g = torch.randn_like(ref)
    y.backward(g.to(y.dtype))
    _grad.join()
    dw_ref = torch.ops.aten.convolution_backward(g, x.float(), c.weight.float(), None, [2, 2], [3, 3], [1, 1],
                                                 False, [0, 0], 1, [False, True, False])[1]
    _close(c.weight.grad, dw_ref, 3e-2, "stem wgrad")


def test_pointwise_dgrad_accumulates_into_shortcut_gradient(monkeypatch):
    """Identity blocks: conv1's backward-data GEMM accumulates into the shortcut gradient the next
    fused BN deposited (beta = 1), so the producing BN reads one gradient tensor. Gradients match
    the separate-tensors path within bf16 rounding."""
    from determined_clone_amd.models import resnet
    from determined_clone_amd.ops import conv as conv_ops

    torch.manual_seed(0)
    # deterministic MIOpen solvers: the two runs then differ only by where the summed gradient is
    # rounded to bf16 (with atomics-based solvers two identical runs differ by ~20% here)
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    dev = torch.device("cuda")
    base = resnet.to_mi355x_layout(resnet.ResNet([2, 2, 1, 1], num_classes=10, zero_init_residual=False)).to(dev)
    x = torch.randn(16, 3, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=dev)
    # the GEMM for every stride-1 backward-data (where the accumulate path applies), MIOpen otherwise
    monkeypatch.setattr(conv_ops, "_choose", lambda key, cands: 1 if key[0] == "dgrad" else 0)
    grads = []
    real_sink = conv_ops._grad_sink
    for acc in (False, True):
        monkeypatch.setattr(conv_ops, "_grad_sink", real_sink if acc else (lambda x: None))
        hits = conv_ops.ACC_HITS
        model = copy.deepcopy(base)
        F.cross_entropy(model(x).float(), y).backward()
        torch.cuda.synchronize()
        grads.append([p.grad.float() for p in model.parameters()])
        if acc:
            assert conv_ops.ACC_HITS - hits == 2  # layer1.1 and layer2.1
    # one extra bf16 rounding of one tensor: ~1% typical (measured 0.6-1.5%, 6% on the stem BN
    # bias whose gradient cancels heavily); a wrong accumulation would be O(1)
    names = [n for n, _ in base.named_parameters()]
    rel = [((a - b).norm() / (a.norm() + 1e-12)).item() for a, b in zip(*grads)]
    assert max(rel) < 0.1, max(zip(rel, names))
    assert sorted(rel)[len(rel) // 2] < 0.02, sorted(rel)[len(rel) // 2]


# ----------------------------------------------------------------------------- implicit GEMM (3x3)
IGEMM_SHAPES = [
    # (N, C, H, K, stride): ResNet-50 3x3 shapes (small batch) + ragged pixel counts
    (2, 64, 56, 64, 1), (2, 128, 56, 128, 2), (3, 128, 28, 128, 1), (2, 256, 28, 256, 2),
    (4, 256, 14, 256, 1), (3, 512, 14, 512, 2), (5, 512, 7, 512, 1), (1, 64, 5, 128, 1),
    (1, 192, 9, 64, 2),
    # ragged last pixel tiles, stride 2, C != K (also ran the removed 8-wave kernel: round6_igemm_big_tile_ab.txt)
    (2, 128, 14, 256, 1), (1, 256, 9, 128, 2), (3, 64, 11, 256, 1), (2, 512, 7, 128, 1),
]


def _igemm_inputs(n, c, h, k, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, c, h, h, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(k, c, 3, 3, generator=g) / (9 * c) ** 0.5).cuda().bfloat16().contiguous(
        memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("shape", IGEMM_SHAPES)
def test_conv_igemm_forward_stats_and_dgrad(shape):
    """Forward + fused BN statistics + stride-1 data gradient vs fp32 convolutions."""
    C = _ext.load()
    n, c, h, k, st = shape
    x, w = _igemm_inputs(n, c, h, k)
    y, partial = C.conv_igemm_fwd(x, w, st, 1, True)
    ref = F.conv2d(x.float(), w.float(), stride=st, padding=1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    _close(y, ref, 1e-2, "y")
    yc = y.float().permute(0, 2, 3, 1).reshape(-1, k)
    got = partial.sum(0)
    torch.testing.assert_close(got[0], yc.sum(0), atol=1e-2 * yc.shape[0] ** 0.5, rtol=1e-3)
    torch.testing.assert_close(got[1], (yc * yc).sum(0), atol=1e-2, rtol=1e-3)
    y2, p2 = C.conv_igemm_fwd(x, w, st, 1, False)
    assert p2 is None
    torch.testing.assert_close(y2, y, atol=0, rtol=0)
    if st == 1:
        g = torch.Generator(device="cpu").manual_seed(1)
        dy = torch.randn(ref.shape, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
        dref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [1, 1], [1, 1],
                                                   [1, 1], False, [0, 0], 1, [True, False, False])[0]
        _close(C.conv_igemm_dgrad(dy, w, 1), dref, 1e-2, "dx")


@pytest.mark.parametrize("ck", [(64, 64), (128, 256), (256, 128)])
def test_conv_igemm_asymmetric_weight_orientation(ck):
    """A weight that is non-zero at ONE tap and ONE (k, c) pair: catches transposed taps /
    swapped channel maps that random data can hide (the 256 x 64 tile at K = 64, 128 x 128 tiles
    with several channel tiles at K = 256 / 128)."""
    C = _ext.load()
    c, k = ck
    x, w = _igemm_inputs(2, c, 9, k)
    w = torch.zeros_like(w)
    w[5, 17, 0, 2] = 1.0  # k=5 reads channel 17 at tap (r=0, s=2)
    w[k - 3, c - 2, 2, 1] = -2.0  # last channel tiles, another tap
    y, _ = C.conv_igemm_fwd(x, w, 1, 1, False)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    torch.testing.assert_close(y.float(), ref, atol=0, rtol=0)
    dy = torch.zeros_like(y)
    dy[0, 5, 4, 4] = 1.0
    dx = C.conv_igemm_dgrad(dy, w, 1)
    dref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [1, 1], [1, 1],
                                               [1, 1], False, [0, 0], 1, [True, False, False])[0]
    torch.testing.assert_close(dx.float(), dref, atol=0, rtol=0)


@pytest.mark.parametrize("stride", [1, 2])
def test_spatial_conv_igemm_autograd_and_bn(stride, monkeypatch):
    """conv3x3 -> fused BN through the model path: output, BN statistics source, input and weight
    gradients (our wgrad kernel) against the fp32 PyTorch composition."""
    monkeypatch.setattr(conv, "IGEMM_WGRAD", "1")
    torch.manual_seed(0)
    conv_m = nn.Conv2d(128, 128, 3, stride=stride, padding=1, bias=False).cuda().bfloat16().to(
        memory_format=torch.channels_last)
    bn = nn.BatchNorm2d(128).cuda()
    x = torch.randn(4, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    assert conv.igemm_supported(conv_m, x)
    y = conv.spatial_conv(conv_m, x, bn_stats=True)
    assert getattr(y, "_dca_bn_partials", None) is not None
    captured = []
    y.register_hook(lambda gr: captured.append(gr))
    out = batchnorm.batch_norm_act(y, bn.weight, bn.bias, bn.running_mean.clone(), bn.running_var.clone(),
                                   training=True, momentum=0.1, eps=1e-5, relu=True)
    g = torch.randn_like(out)
    out.backward(g)
    x32 = x.detach().float()
    w32 = conv_m.weight.detach().float()
    ref = F.relu(F.batch_norm(F.conv2d(x32, w32, stride=stride, padding=1), None, None, bn.weight.float(),
                              bn.bias.float(), training=True, eps=1e-5))
    _close(out, ref, 3e-2, "bn(conv(x))")
    # the convolution's own backward, fed the gradient that reached its output (the BN backward
    # in bf16 is checked by the batchnorm tests; its mean-subtraction cancels too much at this
    # small batch for an end-to-end fp32 comparison of dW)
    (dy,) = captured
    dref = torch.ops.aten.convolution_backward(dy.float(), x32, w32, None, [stride, stride], [1, 1], [1, 1],
                                               False, [0, 0], 1, [True, True, False])
    _close(x.grad, dref[0], 1e-2, "dx")
    _close(conv_m.weight.grad, dref[1], 1e-2, "dw")


@pytest.mark.parametrize("k,stride", [(3, 1), (3, 2), (1, 1), (1, 2)])
def test_conv_igemm_wgrad_accumulates_into_grad_views(k, stride):
    """dW added into an existing fp32 .grad in both layouts the optimizers use: channels_last
    (the parameter's own) and contiguous NCHW (a flat-buffer view)."""
    C = _ext.load()
    torch.manual_seed(0)
    x = torch.randn(2, 128, 14, 14, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 128, k, k, device="cuda") / (k * k * 128) ** 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last)
    pad = k // 2
    y = F.conv2d(x.float(), w.float(), stride=stride, padding=pad)
    dy = torch.randn_like(y).bfloat16().contiguous(memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [stride, stride],
                                              [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    for fmt in (torch.channels_last, torch.contiguous_format):
        base = torch.randn(w.shape, device="cuda").contiguous(memory_format=fmt)
        acc = base.clone()
        out = C.conv_igemm_wgrad(dy, x, w, stride, pad, acc)
        assert out.data_ptr() == acc.data_ptr()
        _close(acc - base, ref, 1e-2, f"dw ({fmt})")


@pytest.mark.parametrize("shape", [(4, 256, 56, 56, 2), (3, 64, 57, 29, 2), (2, 1024, 14, 14, 2), (2, 128, 9, 9, 3)])
def test_strided_accumulate_matches_strided_add(shape):
    """dx[:, :, s*i, s*j] += small[:, :, i, j] (the projection shortcut's data gradient of a
    downsampling block) on the HIP kernel equals ATen's strided add bit for bit (fp32 add of two
    bf16 values, one rounding)."""
    from determined_clone_amd.ops import _ext

    n, c, h, w, s = shape
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    torch.manual_seed(0)
    dx = torch.randn(n, c, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    small = torch.randn(n, c, ho, wo, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    want = dx.clone()
    want[:, :, ::s, ::s] += small
    _ext.load().strided_accumulate(dx, small, s)
    torch.testing.assert_close(dx, want, atol=0, rtol=0)
