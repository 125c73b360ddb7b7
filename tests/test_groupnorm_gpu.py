"""Fused NHWC GroupNorm(+SiLU) HIP kernels vs the fp32 PyTorch oracle (forward, input gradient,
affine gradients returned or accumulated into persistent .grad views)."""
import pytest
import torch
import torch.nn.functional as F

from determined_clone_amd.ops import groupnorm as gn

pytestmark = pytest.mark.gpu


def _ref(x, w, b, G, eps, act):
    y = F.group_norm(x, G, w, b, eps)
    return F.silu(y) if act else y


@pytest.mark.parametrize("N,C,H,G,act,dtype", [
    (2, 320, 16, 32, True, torch.bfloat16), (2, 640, 8, 32, True, torch.bfloat16),
    (3, 64, 12, 32, False, torch.bfloat16), (2, 1280, 4, 32, True, torch.float32),
    (1, 128, 64, 8, True, torch.bfloat16)])
def test_groupnorm_matches_fp32(N, C, H, G, act, dtype):
    torch.manual_seed(0)
    x = (torch.randn(N, C, H, H, device="cuda") * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
    b = (torch.randn(C, device="cuda") * 0.1).requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    y = gn.group_norm_act(xg, G, w, b, 1e-5, act)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.float().detach().requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    yr = _ref(xr, wr, br, G, 1e-5, act)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, rtol=tol, atol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    torch.testing.assert_close(xg.grad.float(), xr.grad, rtol=5 * tol, atol=5 * tol)
    torch.testing.assert_close(w.grad, wr.grad, rtol=5 * tol, atol=5 * tol * N * H * H ** 0.5)
    torch.testing.assert_close(b.grad, br.grad, rtol=5 * tol, atol=5 * tol * N * H * H ** 0.5)


def test_groupnorm_accumulates_into_flat_grads():
    from determined_clone_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(1)
    m = gn.GroupNormAct(32, 320, act=True).cuda()
    FlatParamSpace([list(m.parameters())])
    x = torch.randn(2, 320, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    m.weight.grad.fill_(1.0)
    m.bias.grad.fill_(2.0)
    m(x).float().sum().backward()
    ref = gn.GroupNormAct(32, 320, act=True).cuda()
    ref.load_state_dict(m.state_dict())
    xr = x.float().contiguous()
    _ref(xr, ref.weight, ref.bias, 32, 1e-5, True).sum().backward()
    torch.testing.assert_close(m.weight.grad, ref.weight.grad + 1.0, rtol=3e-2, atol=0.5)
    torch.testing.assert_close(m.bias.grad, ref.bias.grad + 2.0, rtol=3e-2, atol=0.5)
