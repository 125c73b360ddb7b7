"""CPU paths of the transformer ops (the fp32 references the GPU kernels are checked against)."""
import torch
import torch.nn.functional as F

from determined_clone_amd.ops import transformer as T


def test_reference_attention_matches_sdpa():
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 17, 3, 16) for _ in range(3))
    for causal in (True, False):
        o = T.flash_attention(q, k, v, causal=causal)
        ref = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                             is_causal=causal).transpose(1, 2)
        torch.testing.assert_close(o, ref, atol=1e-5, rtol=1e-5)


def test_rope_is_rotation_and_inverse():
    torch.manual_seed(1)
    x = torch.randn(2, 9, 2, 8)
    cos, sin = T.rope_tables(16, 8)
    y = T.rope(x, cos, sin)
    torch.testing.assert_close(y.norm(dim=-1), x.norm(dim=-1), atol=1e-5, rtol=1e-5)
    # position 0 is the identity
    torch.testing.assert_close(y[:, 0], x[:, 0])
    # rotating by -theta undoes it
    back = T.reference_rope(y, cos, -sin)
    torch.testing.assert_close(back, x, atol=1e-5, rtol=1e-5)


def test_layer_norm_residual_returns_sum():
    torch.manual_seed(2)
    x, r = torch.randn(4, 32), torch.randn(4, 32)
    w, b = torch.rand(32), torch.randn(32)
    y, s = T.layer_norm(x, w, b, 1e-5, residual=r)
    torch.testing.assert_close(s, x + r)
    torch.testing.assert_close(y, F.layer_norm(x + r, (32,), w, b, 1e-5))


def test_bias_gelu_reference():
    x, b = torch.randn(3, 8), torch.randn(8)
    torch.testing.assert_close(T.bias_gelu(x, b), F.gelu(x + b, approximate="tanh"))
