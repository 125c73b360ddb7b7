"""Numerics of the HIP kernels vs plain PyTorch fp32 references (run on an MI355X)."""
import pytest
import torch

from determined_clone_amd.ops import _ext, batchnorm
from determined_clone_amd.ops import optim as fopt

pytestmark = pytest.mark.gpu


def _ext_loaded():
    C = _ext.load()
    assert C.__file__.endswith("_C.so")
    return C


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 64, 14, 14), (4, 256, 7, 7), (2, 2048, 3, 3), (16, 24, 5, 5),
                                   (32, 128, 28, 28), (3, 64, 17, 19)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_forward_backward(dtype, shape, relu, res):
    _ext_loaded()
    torch.manual_seed(0)
    N, C, H, W = shape
    dev = "cuda"
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    r = torch.randn(shape, device=dev).to(dtype).contiguous(memory_format=torch.channels_last) if res else None
    w = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    x1 = x.clone().requires_grad_(True)
    w1, b1 = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    r1 = r.clone().requires_grad_(True) if res else None
    y = batchnorm.batch_norm_act(x1, w1, b1, rm, rv, residual=r1, training=True, momentum=0.1,
                                 eps=1e-5, relu=relu, num_batches_tracked=nbt)
    # fp32 reference
    x2 = x.float().clone().requires_grad_(True)
    w2, b2 = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    r2 = r.float().clone().requires_grad_(True) if res else None
    rm2, rv2 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y2 = batchnorm.reference_batch_norm_act(x2, w2, b2, rm2, rv2, r2, True, 0.1, 1e-5, relu)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), y2, atol=tol * 4, rtol=tol)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(rv, rv2, atol=1e-3, rtol=1e-3)
    assert int(nbt) == (1 if C % 8 == 0 else 1)
    g = torch.randn_like(y2)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    y2.backward(g)
    # bf16 grads: compare against the fp32 reference computed from the same rounded inputs
    torch.testing.assert_close(x1.grad.float(), x2.grad, atol=tol * 10, rtol=tol * 5)
    torch.testing.assert_close(w1.grad, w2.grad, atol=tol * 50, rtol=tol * 5)
    torch.testing.assert_close(b1.grad, b2.grad, atol=tol * 50, rtol=tol * 5)
    if res:
        torch.testing.assert_close(r1.grad.float(), r2.grad, atol=tol * 4, rtol=tol)


def test_bn_eval_affine():
    _ext_loaded()
    x = torch.randn(4, 64, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w, b = torch.rand(64, device="cuda"), torch.randn(64, device="cuda")
    rm, rv = torch.randn(64, device="cuda"), torch.rand(64, device="cuda") + 0.5
    with torch.no_grad():
        y = batchnorm.batch_norm_act(x, w, b, rm, rv, training=False, relu=True)
        y2 = batchnorm.reference_batch_norm_act(x.float(), w, b, rm, rv, None, False, 0.1, 1e-5, True)
    torch.testing.assert_close(y.float(), y2, atol=3e-2, rtol=2e-2)


def _params(dtype):
    torch.manual_seed(1)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda").to(dtype)) for s in [(37,), (64, 3, 3, 3), (1000, 17), (5,)]]
    return ps


@pytest.mark.parametrize("kind", ["sgd", "sgd_nesterov", "adam", "adamw"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_optimizers_match_torch(kind, dtype):
    _ext_loaded()
    ps = _params(dtype)
    ref = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]
    if kind.startswith("sgd"):
        kw = dict(lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=kind == "sgd_nesterov")
        fused = fopt.FusedSGD(ps, **kw)
        tref = torch.optim.SGD(ref, **kw)
    elif kind == "adam":
        fused = fopt.FusedAdam(ps, lr=1e-2, weight_decay=1e-3)
        tref = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-3)
    else:
        fused = fopt.FusedAdamW(ps, lr=1e-2, weight_decay=1e-2)
        tref = torch.optim.AdamW(ref, lr=1e-2, weight_decay=1e-2)
    for step in range(4):
        grads = [torch.randn(p.shape, device="cuda") for p in ps]
        for p, g in zip(ps, grads):
            p.grad.copy_(g.to(dtype))
        for p, g in zip(ref, grads):
            p.grad = g.to(dtype).float()
        fused.step()
        tref.step()
    for st in fused.flat.values():
        for seg in st.buf.segments:
            got = st.buf.view(st.master, seg)
            want = ref[seg.index].detach()
            torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)
            torch.testing.assert_close(seg.param.detach().float(), want, atol=2e-2, rtol=1e-2)


def test_grad_clip_and_found_inf():
    _ext_loaded()
    ps = _params(torch.float32)
    opt = fopt.FusedSGD(ps, lr=1.0)
    for p in ps:
        p.grad.fill_(1.0)
    n = sum(p.numel() for p in ps)
    before = [p.detach().clone() for p in ps]
    opt.prepare_grads(max_norm=1.0)
    assert abs(float(opt.last_grad_norm) - n ** 0.5) / n ** 0.5 < 1e-5
    opt.step()
    delta = torch.cat([(b - p.detach()).flatten() for b, p in zip(before, ps)])
    assert abs(float(delta.norm()) - 1.0) < 1e-4
    # inf gradient -> step skipped
    ps[0].grad[0] = float("inf")
    snap = [p.detach().clone() for p in ps]
    opt.prepare_grads(max_norm=1.0)
    assert float(opt.found_inf) == 1.0
    opt.step()
    for s, p in zip(snap, ps):
        assert torch.equal(s, p.detach())


def test_lamb_matches_reference():
    _ext_loaded()
    ps = _params(torch.float32)
    ref = [torch.nn.Parameter(p.detach().clone().cpu()) for p in ps]
    f = fopt.FusedLAMB(ps, lr=1e-2, weight_decay=0.01)
    r = fopt.FusedLAMB(ref, lr=1e-2, weight_decay=0.01)  # CPU path = reference math
    for _ in range(3):
        grads = [torch.randn(p.shape) for p in ps]
        for p, g in zip(ps, grads):
            p.grad.copy_(g.cuda())
        for p, g in zip(ref, grads):
            p.grad.copy_(g)
        f.step()
        r.step()
    for p, q in zip(ps, ref):
        torch.testing.assert_close(p.detach().cpu(), q.detach(), atol=1e-5, rtol=1e-4)


def test_device_grad_scaler():
    _ext_loaded()
    ps = _params(torch.float32)
    opt = fopt.FusedSGD(ps, lr=0.1)
    sc = fopt.DeviceGradScaler(init_scale=1024.0, growth_interval=1)
    for p in ps:
        p.grad.fill_(1024.0)
    before = [p.detach().clone() for p in ps]
    sc.step(opt)
    sc.update()
    assert sc.get_scale() == 2048.0
    for b, p in zip(before, ps):
        torch.testing.assert_close(b - p.detach(), torch.full_like(b, 0.1))
    ps[1].grad.fill_(float("nan"))
    sc.step(opt)
    sc.update()
    assert sc.get_scale() == 1024.0


def test_resnet_residual_grad_sink_matches_autograd_add():
    """Identity-shortcut gradients summed inside the producer BN kernel (ResidualGradSink) equal
    the plain autograd add path."""
    _ext_loaded()
    from determined_clone_amd.models import resnet

    torch.manual_seed(0)
    m1 = resnet.ResNet([2, 2, 1, 1], num_classes=10).cuda().to(memory_format=torch.channels_last)
    m2 = resnet.ResNet([2, 2, 1, 1], num_classes=10).cuda().to(memory_format=torch.channels_last)
    m2.load_state_dict(m1.state_dict())
    for blk in m2.modules():
        if isinstance(blk, resnet.Bottleneck):
            blk.forward = (lambda self: (lambda x: self.bn3(self.conv3(self.bn2(self.conv2(self.bn1(self.conv1(x))))),
                                                             residual=x if self.downsample is None else self.downsample(x))))(blk)
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    for m in (m1, m2):
        m(x).float().square().mean().backward()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(a.grad, b.grad, atol=1e-5, rtol=1e-4, msg=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hw", [(16, 16), (15, 13), (112, 112)])
def test_bn_relu_maxpool_stem(dtype, hw):
    _ext_loaded()
    torch.manual_seed(0)
    N, C = (4, 64) if hw[0] < 100 else (2, 64)
    x = torch.randn(N, C, *hw, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda") * 0.5
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    x1, w1, b1 = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = batchnorm.batch_norm_relu_maxpool(x1, w1, b1, rm, rv, training=True, momentum=0.1, eps=1e-5)
    x2, w2, b2 = x.float().clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y2 = batchnorm.reference_bn_relu_maxpool(x2, w2, b2, rm2, rv2, True, 0.1, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), y2, atol=tol * 4, rtol=tol)
    torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
    g = torch.randn_like(y2)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    y2.backward(g)
    rel = lambda a, r: ((a.float() - r).norm() / r.norm()).item()  # noqa: E731
    assert rel(x1.grad, x2.grad) < (3e-2 if dtype == torch.bfloat16 else 1e-4)
    assert rel(w1.grad, w2.grad) < 1e-2 and rel(b1.grad, b2.grad) < 1e-2
    # eval path
    y3 = batchnorm.batch_norm_relu_maxpool(x, w, b, rm, rv, training=False, eps=1e-5)
    y4 = batchnorm.reference_bn_relu_maxpool(x.float(), w, b, rm, rv, False, 0.1, 1e-5)
    torch.testing.assert_close(y3.float(), y4, atol=tol * 4, rtol=tol)


def test_bn_direct_grad_accumulation_into_flat_buffer():
    """BN weight/bias grads accumulated in-kernel into FlatParamSpace .grad views equal autograd's
    AccumulateGrad path over two backward passes, and post-accumulate hooks (DDP/ZeRO triggers)
    still fire once per backward."""
    _ext_loaded()
    from determined_clone_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    C = 64
    x = torch.randn(8, C, 10, 10, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(8, C, 10, 10, device="cuda")
    w1 = torch.nn.Parameter(torch.rand(C, device="cuda") + 0.5)
    b1 = torch.nn.Parameter(torch.randn(C, device="cuda"))
    w2 = torch.nn.Parameter(w1.detach().clone())
    b2 = torch.nn.Parameter(b1.detach().clone())
    space = FlatParamSpace([[w1, b1]])
    assert w1._dca_direct_grad and w1.grad is not None
    calls = []
    w1.register_post_accumulate_grad_hook(lambda p: calls.append("w"))
    b1.register_post_accumulate_grad_hook(lambda p: calls.append("b"))
    ptr = w1.grad.data_ptr()
    for w, b in ((w1, b1), (w2, b2)):
        for _ in range(2):
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            y = batchnorm.batch_norm_act(x, w, b, rm, rv)
            (y.float() * g).sum().backward()
    assert w1.grad.data_ptr() == ptr  # still the flat view
    assert sorted(calls) == ["b", "b", "w", "w"]
    torch.testing.assert_close(w1.grad, w2.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(b1.grad, b2.grad, atol=1e-3, rtol=1e-4)
    assert space.grads_are_views()


def test_global_avg_pool_matches_torch():
    _ext_loaded()
    torch.manual_seed(0)
    x = torch.randn(6, 64, 7, 7, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    y = batchnorm.global_avg_pool(x1)
    x2 = x.float().clone().requires_grad_(True)
    y2 = torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x2, 1), 1)
    torch.testing.assert_close(y.float(), y2, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(y2)
    y.backward(g.bfloat16())
    y2.backward(g)
    assert x1.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x1.grad.float(), x2.grad, atol=1e-3, rtol=1e-2)


def _bn_pair(C, dev, seed):
    from determined_clone_amd.models.resnet import BatchNormAct2d

    g = torch.Generator(device="cpu").manual_seed(seed)
    a = BatchNormAct2d(C, relu=True).to(dev)
    b = BatchNormAct2d(C, relu=False).to(dev)
    with torch.no_grad():
        for m in (a, b):
            m.weight.copy_(torch.rand(C, generator=g) + 0.5)
            m.bias.copy_(torch.randn(C, generator=g))
    return a, b


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 256, 14, 14), (4, 512, 7, 7), (2, 2048, 3, 3), (3, 64, 17, 19)])
@pytest.mark.parametrize("with_partials,with_dy2", [(False, False), (True, True)])
def test_bn_act_dual_matches_fp32(dtype, shape, with_partials, with_dy2):
    """relu(bn3(x) + bn_ds(x2)) (a downsampling block's tail, csrc/batchnorm.hip *_dual) against
    two fp32 BatchNorms + add + ReLU: output, running statistics of BOTH BatchNorms, gradients of
    both inputs and all four affine parameters; with statistics partials supplied by a producer
    and an extra upstream gradient deposited by a consumer (dy2)."""
    _ext_loaded()
    torch.manual_seed(0)
    N, C, H, W = shape
    dev = "cuda"
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    x2 = (torch.randn(shape, device=dev) * 0.7 - 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    bn, bnd = _bn_pair(C, dev, 1)
    rbn, rbnd = _bn_pair(C, dev, 1)
    xa, x2a = x.clone().requires_grad_(True), x2.clone().requires_grad_(True)
    if with_partials:  # the convolution epilogue's [blocks, 2, C] (sum, sum^2) layout
        for t, src in ((xa, x), (x2a, x2)):
            rows = src.float().permute(0, 2, 3, 1).reshape(-1, C)
            parts = torch.stack([torch.stack([r.sum(0), (r * r).sum(0)]) for r in rows.chunk(3)])
            t._dca_bn_partials = parts.contiguous()
    y = batchnorm.batch_norm_act_dual(xa, bn, x2a, bnd)
    xr, x2r = x.float().clone().requires_grad_(True), x2.float().clone().requires_grad_(True)
    yr = batchnorm.reference_batch_norm_act_dual(xr, rbn, x2r, rbnd)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol * 4, rtol=tol)
    for m, r in ((bn, rbn), (bnd, rbnd)):
        torch.testing.assert_close(m.running_mean, r.running_mean, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(m.running_var, r.running_var, atol=1e-3, rtol=1e-3)
        assert int(m.num_batches_tracked) == 1
    g = torch.randn_like(yr)
    extra = torch.randn_like(yr) if with_dy2 else None
    if with_dy2:  # a consumer deposits a second upstream gradient into the output's sink
        y._dca_grad_sink.deposit(extra.to(dtype).contiguous(memory_format=torch.channels_last))
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    yr.backward(g + extra if with_dy2 else g)
    torch.testing.assert_close(xa.grad.float(), xr.grad, atol=tol * 10, rtol=tol * 5)
    torch.testing.assert_close(x2a.grad.float(), x2r.grad, atol=tol * 10, rtol=tol * 5)
    for m, r in ((bn, rbn), (bnd, rbnd)):
        torch.testing.assert_close(m.weight.grad, r.weight.grad, atol=tol * 50, rtol=tol * 5)
        torch.testing.assert_close(m.bias.grad, r.bias.grad, atol=tol * 50, rtol=tol * 5)


def test_resnet_downsample_block_dual_bn_matches_separate(monkeypatch):
    """A bf16 ResNet stage whose downsampling block runs the fused dual BatchNorm gives the same
    output and gradients as the same block with two separate BatchNorms (DCA_BN_DUAL=0 path)."""
    from determined_clone_amd.models import resnet

    _ext_loaded()
    torch.manual_seed(0)
    blk = resnet.Bottleneck(256, 128, stride=2)
    blk = resnet.to_mi355x_layout(blk).cuda()
    x = torch.randn(8, 256, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for dual in (True, False):
        monkeypatch.setattr(resnet, "BN_DUAL", dual)
        for p in blk.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        y = blk(xi)
        y.float().square().mean().backward()
        outs.append((y.float(), xi.grad.float(), {n: p.grad.float().clone() for n, p in blk.named_parameters()}))
    (y1, g1, p1), (y2, g2, p2) = outs
    torch.testing.assert_close(y1, y2, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(g1, g2, atol=5e-3, rtol=5e-2)
    for n in p1:
        torch.testing.assert_close(p1[n], p2[n], atol=5e-3, rtol=5e-2, msg=n)
