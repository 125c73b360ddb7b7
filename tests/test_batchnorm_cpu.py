"""CPU semantics of the fused BatchNorm ops' fallback paths against torch's own BatchNorm2d
(the GPU kernels are compared against the same references in tests/test_ops_gpu.py)."""
import torch
import torch.nn as nn

from determined_clone_amd.ops import batchnorm as B


def _pair(momentum):
    torch.manual_seed(0)
    a, b = nn.BatchNorm2d(8, momentum=momentum), nn.BatchNorm2d(8, momentum=momentum)
    for m in (a, b):
        m.weight.data.uniform_(0.5, 1.5)
        m.bias.data.uniform_(-0.5, 0.5)
    ra, rb = nn.BatchNorm2d(8, momentum=momentum), nn.BatchNorm2d(8, momentum=momentum)
    ra.load_state_dict(a.state_dict())
    rb.load_state_dict(b.state_dict())
    return a, b, ra, rb


def test_dual_bn_cumulative_average_momentum_none():
    """``batch_norm_act_dual`` with ``momentum=None`` keeps torch's cumulative moving
    average (1 / num_batches_tracked) instead of freezing the running statistics."""
    a, b, ra, rb = _pair(None)
    for step in range(4):
        x, x2 = torch.randn(4, 8, 5, 5) + step, torch.randn(4, 8, 5, 5) * (step + 1)
        y = B.batch_norm_act_dual(x, a, x2, b)
        yr = torch.relu(ra(x) + rb(x2))
        torch.testing.assert_close(y, yr)
    for m, r in ((a, ra), (b, rb)):
        torch.testing.assert_close(m.running_mean, r.running_mean)
        torch.testing.assert_close(m.running_var, r.running_var)
        assert int(m.num_batches_tracked) == int(r.num_batches_tracked) == 4
    assert not torch.allclose(a.running_mean, torch.zeros(8))


def test_dual_bn_fixed_momentum_and_eval():
    a, b, ra, rb = _pair(0.1)
    x, x2 = torch.randn(4, 8, 5, 5), torch.randn(4, 8, 5, 5)
    torch.testing.assert_close(B.batch_norm_act_dual(x, a, x2, b), torch.relu(ra(x) + rb(x2)))
    for m in (a, b, ra, rb):
        m.eval()
    torch.testing.assert_close(B.batch_norm_act_dual(x, a, x2, b), torch.relu(ra(x) + rb(x2)))


def test_single_bn_momentum_none_matches_torch():
    torch.manual_seed(1)
    m, r = nn.BatchNorm2d(8, momentum=None), nn.BatchNorm2d(8, momentum=None)
    for step in range(3):
        x = torch.randn(2, 8, 4, 4) * (step + 1)
        y = B.batch_norm_act(x, m.weight, m.bias, m.running_mean, m.running_var, momentum=None,
                             num_batches_tracked=m.num_batches_tracked)
        torch.testing.assert_close(y, torch.relu(r(x)))
    torch.testing.assert_close(m.running_var, r.running_var)
