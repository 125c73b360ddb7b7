"""CPU paths of the transformer ops (the fp32 references the GPU kernels are checked against)."""
import pytest
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


def test_reference_attention_key_lengths_match_additive_mask():
    torch.manual_seed(11)
    B, S, H, D = 3, 10, 2, 8
    q, k, v = (torch.randn(B, S, H, D) for _ in range(3))
    lens = torch.tensor([10, 4, 1])
    o = T.reference_attention(q, k, v, causal=False, key_lengths=lens)
    add = torch.where(torch.arange(S)[None] < lens[:, None], 0.0, float("-inf"))[:, None, None, :]
    ref = torch.nn.functional.scaled_dot_product_attention(
        q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), attn_mask=add).transpose(1, 2)
    torch.testing.assert_close(o, ref, atol=1e-5, rtol=1e-5)
    # CPU flash_attention routes to the same reference
    torch.testing.assert_close(T.flash_attention(q, k, v, causal=False, key_lengths=lens), o)


def test_hf_mask_to_key_lengths():
    from determined_clone_amd.transformers import mask_to_key_lengths

    S = 6
    lens = torch.tensor([6, 3, 1])
    pad = torch.arange(S)[None] < lens[:, None]
    m = pad[:, None, None, :].expand(3, 1, S, S).clone()
    assert mask_to_key_lengths(m, causal=False).tolist() == [6, 3, 1]
    assert mask_to_key_lengths(m, causal=True) is None  # not causal-shaped
    mc = m & torch.ones(S, S, dtype=torch.bool).tril()
    assert mask_to_key_lengths(mc, causal=True).tolist() == [6, 3, 1]
    left = pad.flip(-1)[:, None, None, :].expand(3, 1, S, S).clone()  # left padding
    assert mask_to_key_lengths(left, causal=False) is None
    empty = m.clone()
    empty[2] = False
    assert mask_to_key_lengths(empty, causal=False) is None


def test_hf_bert_on_cpu_falls_back_to_sdpa():
    transformers = pytest.importorskip("transformers")
    from determined_clone_amd.transformers import use_flash_attention

    torch.manual_seed(12)
    cfg = transformers.BertConfig(vocab_size=100, hidden_size=128, num_hidden_layers=1,
                                  num_attention_heads=2, intermediate_size=256)
    a, b = transformers.BertModel(cfg).eval(), transformers.BertModel(cfg).eval()
    b.load_state_dict(a.state_dict())
    a.set_attn_implementation("sdpa")
    use_flash_attention(b)
    ids = torch.randint(1, 100, (2, 12))
    mask = torch.ones(2, 12, dtype=torch.long)
    mask[1, 5:] = 0
    with torch.no_grad():
        torch.testing.assert_close(b(input_ids=ids, attention_mask=mask).last_hidden_state,
                                   a(input_ids=ids, attention_mask=mask).last_hidden_state)


def test_reference_attention_grouped_query_matches_sdpa_gqa():
    """K/V with fewer heads (GQA / MQA): query head h reads K/V head h // (H / Hkv)."""
    torch.manual_seed(12)
    B, S, H, Hkv, D = 2, 9, 6, 2, 8
    q = torch.randn(B, S, H, D)
    k, v = (torch.randn(B, S, Hkv, D) for _ in range(2))
    for causal in (True, False):
        o = T.flash_attention(q, k, v, causal=causal)
        ref = F.scaled_dot_product_attention(
            q.transpose(1, 2), k.repeat_interleave(H // Hkv, 2).transpose(1, 2),
            v.repeat_interleave(H // Hkv, 2).transpose(1, 2), is_causal=causal).transpose(1, 2)
        torch.testing.assert_close(o, ref, atol=1e-5, rtol=1e-5)
