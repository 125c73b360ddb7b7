"""Numerics of the transformer HIP kernels (LayerNorm, bias+GELU, RoPE, MFMA flash attention)
against plain PyTorch fp32 references (run on an MI355X)."""
import copy
import math

import pytest
import torch

from determined_clone_amd.ops import _ext
from determined_clone_amd.ops import transformer as T

pytestmark = pytest.mark.gpu


def _C():
    C = _ext.load()
    assert C.__file__.endswith("_C.so")
    return C


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [64, 1024, 1000 - 1000 % 8, 4096])
@pytest.mark.parametrize("res", [False, True])
def test_layer_norm(dtype, D, res):
    _C()
    torch.manual_seed(0)
    rows = 333
    x = (torch.randn(rows, D, device="cuda") * 3 + 1).to(dtype)
    r = torch.randn(rows, D, device="cuda").to(dtype) if res else None
    w = torch.rand(D, device="cuda") + 0.5
    b = torch.randn(D, device="cuda")
    xs = [t.clone().requires_grad_(True) if t is not None else None for t in (x, r, w, b)]
    xr = [t.float().clone().requires_grad_(True) if t is not None else None for t in (x, r, w, b)]
    out = T.layer_norm(xs[0], xs[2], xs[3], 1e-5, residual=xs[1])
    ref = T.reference_layer_norm(xr[0], xr[2], xr[3], 1e-5, residual=xr[1])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    if res:
        y, s = out
        y2, s2 = ref
        torch.testing.assert_close(s.float(), s2, atol=tol, rtol=tol)
        gy, gs = torch.randn_like(y2), torch.randn_like(s2)
        torch.autograd.backward([y, s], [gy.to(dtype), gs.to(dtype)])
        torch.autograd.backward([y2, s2], [gy, gs])
    else:
        y, y2 = out, ref
        gy = torch.randn_like(y2)
        y.backward(gy.to(dtype))
        y2.backward(gy)
    torch.testing.assert_close(y.float(), y2, atol=tol * 4, rtol=tol)
    assert _rel(xs[0].grad, xr[0].grad) < (2e-2 if dtype == torch.bfloat16 else 1e-4)
    if res:
        assert _rel(xs[1].grad, xr[1].grad) < (2e-2 if dtype == torch.bfloat16 else 1e-4)
    assert _rel(xs[2].grad, xr[2].grad) < 1e-2
    assert _rel(xs[3].grad, xr[3].grad) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N", [64, 4096, 1032])
def test_bias_gelu(dtype, N):
    _C()
    torch.manual_seed(1)
    x = torch.randn(257, N, device="cuda").to(dtype)
    b = torch.randn(N, device="cuda") * 0.5
    x1, b1 = x.clone().requires_grad_(True), b.clone().requires_grad_(True)
    x2, b2 = x.float().clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = T.bias_gelu(x1, b1)
    y2 = T.reference_bias_gelu(x2, b2)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), y2, atol=tol, rtol=tol)
    g = torch.randn_like(y2)
    y.backward(g.to(dtype))
    y2.backward(g)
    assert _rel(x1.grad, x2.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
    assert _rel(b1.grad, b2.grad) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rot", [64, 16])
def test_rope(dtype, rot):
    _C()
    torch.manual_seed(2)
    B, S, H, D = 2, 37, 4, 64
    cos, sin = T.rope_tables(64, rot, device="cuda")
    x = torch.randn(B, S, H, D, device="cuda").to(dtype)
    x1 = x.clone().requires_grad_(True)
    x2 = x.float().clone().requires_grad_(True)
    y = T.rope(x1, cos, sin, rot)
    y2 = T.reference_rope(x2, cos, sin, rot)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), y2, atol=tol, rtol=tol)
    g = torch.randn_like(y2)
    y.backward(g.to(dtype))
    y2.backward(g)
    torch.testing.assert_close(x1.grad.float(), x2.grad, atol=tol, rtol=tol)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S", [64, 200, 512])
def test_flash_attention(D, causal, S):
    _C()
    torch.manual_seed(3)
    B, H = 2, 3
    q, k, v = (torch.randn(B, S, H, D, device="cuda").bfloat16() for _ in range(3))
    qs = [t.clone().requires_grad_(True) for t in (q, k, v)]
    qr = [t.float().clone().requires_grad_(True) for t in (q, k, v)]
    o = T.flash_attention(*qs, causal=causal)
    o2 = T.reference_attention(*qr, causal=causal)
    assert _rel(o, o2) < 1e-2, _rel(o, o2)
    g = torch.randn_like(o2)
    o.backward(g.bfloat16())
    o2.backward(g)
    for a, b in zip(qs, qr):
        assert _rel(a.grad, b.grad) < 2e-2, _rel(a.grad, b.grad)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("Sq,Sk", [(300, 300), (77, 300), (512, 129)])
def test_flash_attention_key_padding(D, causal, Sq, Sk):
    """Per-row key lengths (right padding): lengths of 1, inside a tile, on a tile boundary and
    the full length; padded keys must get exactly zero dK / dV."""
    if causal and Sq != Sk:
        pytest.skip("causal needs Sq == Sk")
    _C()
    torch.manual_seed(6)
    B, H = 4, 2
    lens = torch.tensor([1, Sk // 2 + 3, min(128, Sk), Sk], device="cuda")
    q = torch.randn(B, Sq, H, D, device="cuda").bfloat16()
    k, v = (torch.randn(B, Sk, H, D, device="cuda").bfloat16() for _ in range(2))
    qs = [t.clone().requires_grad_(True) for t in (q, k, v)]
    qr = [t.float().clone().requires_grad_(True) for t in (q, k, v)]
    o = T.flash_attention(*qs, causal=causal, key_lengths=lens)
    o2 = T.reference_attention(*qr, causal=causal, key_lengths=lens)
    assert _rel(o, o2) < 1e-2, _rel(o, o2)
    g = torch.randn_like(o2)
    o.backward(g.bfloat16())
    o2.backward(g)
    for a, b in zip(qs, qr):
        assert _rel(a.grad, b.grad) < 2e-2, _rel(a.grad, b.grad)
    for b_, L in enumerate(lens.tolist()):
        if L < Sk:
            assert qs[1].grad[b_, L:].abs().max().item() == 0
            assert qs[2].grad[b_, L:].abs().max().item() == 0


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("H,Hkv", [(8, 2), (6, 1), (4, 4)])
def test_flash_attention_grouped_query(D, causal, H, Hkv):
    """Grouped-query / multi-query attention: K/V with Hkv heads shared by H / Hkv query heads
    each; dK / dV are the sums over each group (fp32 reference through repeat_interleave)."""
    _C()
    torch.manual_seed(8)
    B, S = 2, 300
    lens = torch.tensor([S, 131], device="cuda")
    q = torch.randn(B, S, H, D, device="cuda").bfloat16()
    k, v = (torch.randn(B, S, Hkv, D, device="cuda").bfloat16() for _ in range(2))
    qs = [t.clone().requires_grad_(True) for t in (q, k, v)]
    qr = [t.float().clone().requires_grad_(True) for t in (q, k, v)]
    o = T.flash_attention(*qs, causal=causal, key_lengths=lens)
    o2 = T.reference_attention(*qr, causal=causal, key_lengths=lens)
    assert o.shape == (B, S, H, D)
    assert _rel(o, o2) < 1e-2, _rel(o, o2)
    g = torch.randn_like(o2)
    o.backward(g.bfloat16())
    o2.backward(g)
    for a, b in zip(qs, qr):
        assert a.grad.shape == b.grad.shape
        assert _rel(a.grad, b.grad) < 2e-2, _rel(a.grad, b.grad)
    assert qs[1].grad[1, 131:].abs().max().item() == 0


def test_flash_attention_key_padding_qkvpacked():
    _C()
    torch.manual_seed(7)
    B, S, H, D = 3, 200, 4, 64
    lens = torch.tensor([200, 64, 130], dtype=torch.int64, device="cuda")
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16().requires_grad_(True)
    o = T.flash_attention_qkvpacked(qkv, causal=False, key_lengths=lens)
    qkv2 = qkv.detach().float().requires_grad_(True)
    o2 = T.reference_attention(*qkv2.unbind(2), causal=False, key_lengths=lens)
    assert _rel(o, o2) < 1e-2
    g = torch.randn_like(o2)
    o.backward(g.bfloat16())
    o2.backward(g)
    assert _rel(qkv.grad, qkv2.grad) < 2e-2


@pytest.mark.parametrize("family", ["bert", "vit", "llama_gqa"])
def test_hf_models_on_flash_attention_match_sdpa(family, monkeypatch):
    """HF BERT with a right-padded attention_mask and ViT (S = 197, no mask) on the
    ``dca_mfma`` attention backend agree with HF's own SDPA path, forward and backward."""
    transformers = pytest.importorskip("transformers")
    from determined_clone_amd.transformers import use_flash_attention

    _C()
    torch.manual_seed(8)
    if family == "bert":
        cfg = transformers.BertConfig(vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                                      num_attention_heads=4, intermediate_size=512,
                                      attention_probs_dropout_prob=0.0, hidden_dropout_prob=0.0)
        make = transformers.BertModel
        ids = torch.randint(1, 1000, (3, 96), device="cuda")
        mask = (torch.arange(96, device="cuda")[None] < torch.tensor([96, 40, 7], device="cuda")[:, None]).long()
        inputs = {"input_ids": ids, "attention_mask": mask}
    elif family == "llama_gqa":  # causal, grouped-query K/V (2 K/V heads for 4 query heads)
        cfg = transformers.LlamaConfig(vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                                       num_attention_heads=4, num_key_value_heads=2,
                                       intermediate_size=512, max_position_embeddings=256)
        make = transformers.LlamaModel
        ids = torch.randint(1, 1000, (3, 96), device="cuda")
        mask = (torch.arange(96, device="cuda")[None] < torch.tensor([96, 40, 7], device="cuda")[:, None]).long()
        inputs = {"input_ids": ids, "attention_mask": mask}
    else:
        cfg = transformers.ViTConfig(image_size=224, patch_size=16, hidden_size=256, num_hidden_layers=2,
                                     num_attention_heads=4, intermediate_size=512,
                                     attention_probs_dropout_prob=0.0, hidden_dropout_prob=0.0)
        make = transformers.ViTModel
        inputs = {"pixel_values": torch.randn(2, 3, 224, 224, device="cuda").bfloat16()}
        mask = None
    # separate config objects: set_attn_implementation writes the model's config, and a shared
    # one would switch the SDPA reference models to the backend under test as well.
    # Judged against an fp32 SDPA model: ours (bf16) must be no worse than HF's own bf16 SDPA path
    # (the query-weight gradient is small and cancellation-heavy, so bf16 alone moves it by several percent).
    ref32 = make(copy.deepcopy(cfg)).cuda().float()
    refb = make(copy.deepcopy(cfg)).cuda().bfloat16()
    ours = make(copy.deepcopy(cfg)).cuda().bfloat16()
    refb.load_state_dict(ref32.state_dict())
    ours.load_state_dict(ref32.state_dict())
    for m in (ref32, refb):
        m.set_attn_implementation("sdpa")
    use_flash_attention(ours)
    outs = []
    calls = []
    orig = T.flash_attention
    monkeypatch.setattr(T, "flash_attention", lambda *a, **k: calls.append(a[1].shape) or orig(*a, **k))
    for m in (ref32, refb, ours):
        kw = dict(inputs)
        if "pixel_values" in kw:
            kw["pixel_values"] = kw["pixel_values"].to(next(m.parameters()).dtype)
        h = m(**kw).last_hidden_state
        keep = mask[..., None].to(h.dtype) if mask is not None else torch.ones_like(h[..., :1])
        (h.float() * keep).square().mean().backward()
        wq = next(p for n, p in m.named_parameters() if n.endswith(("query.weight", "q_proj.weight")))
        outs.append((h.float() * keep, wq.grad.float()))
    for k_ in range(2):
        err_sdpa, err_ours = _rel(outs[1][k_], outs[0][k_]), _rel(outs[2][k_], outs[0][k_])
        assert err_ours < max(2 * err_sdpa, 2e-2), (k_, err_ours, err_sdpa)
    assert len(calls) == cfg.num_hidden_layers  # every layer ran on the MFMA kernels (no SDPA fallback)
    if family == "llama_gqa":
        assert calls[0][2] == 2  # K/V passed with their own 2 heads (no repeat)


def test_flash_attention_strided_qkv_slices():
    """Operands sliced from a fused QKV projection output [B, S, 3, H, D] need no copies."""
    _C()
    torch.manual_seed(4)
    B, S, H, D = 2, 128, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16().requires_grad_(True)
    q, k, v = qkv.unbind(2)
    o = T.flash_attention(q, k, v, causal=True)
    qkv2 = qkv.detach().float().requires_grad_(True)
    o2 = T.reference_attention(*qkv2.unbind(2), causal=True)
    assert _rel(o, o2) < 1e-2
    g = torch.randn_like(o2)
    o.backward(g.bfloat16())
    o2.backward(g)
    assert _rel(qkv.grad, qkv2.grad) < 2e-2


def test_flash_attention_matches_sdpa_speed_sanity():
    """Not a benchmark: runs a GPT-2-medium-shaped attention to make sure big grids execute."""
    _C()
    B, S, H, D = 8, 1024, 16, 64
    q, k, v = (torch.randn(B, S, H, D, device="cuda").bfloat16() for _ in range(3))
    o = T.flash_attention(q, k, v, causal=True)
    ref = torch.nn.functional.scaled_dot_product_attention(
        q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True).transpose(1, 2)
    assert _rel(o, ref) < 1e-2
    assert math.isfinite(o.float().abs().max().item())


def test_flash_attention_qkvpacked_matches_unpacked():
    _C()
    torch.manual_seed(5)
    B, S, H, D = 2, 192, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda").bfloat16().requires_grad_(True)
    o = T.flash_attention_qkvpacked(qkv, causal=True)
    qkv2 = qkv.detach().clone().requires_grad_(True)
    o2 = T.flash_attention(*qkv2.unbind(2), causal=True)
    torch.testing.assert_close(o, o2)
    g = torch.randn_like(o)
    o.backward(g)
    o2.backward(g)
    torch.testing.assert_close(qkv.grad, qkv2.grad)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_fused_cross_entropy(dtype):
    _C()
    torch.manual_seed(6)
    N, V = 300, 50304
    logits = (torch.randn(N, V, device="cuda") * 3).to(dtype)
    t = torch.randint(0, 50257, (N,), device="cuda")
    t[::7] = -100
    a = logits.clone().requires_grad_(True)
    b = logits.float().clone().requires_grad_(True)
    la = T.cross_entropy(a, t)
    lb = torch.nn.functional.cross_entropy(b, t, ignore_index=-100)
    torch.testing.assert_close(la, lb, atol=1e-3, rtol=1e-4)
    (la * 3.0).backward()
    (lb * 3.0).backward()
    assert _rel(a.grad, b.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,N", [(1, 8), (333, 1024), (100, 520), (8192, 3072), (4097, 4096), (65536, 1024)])
def test_bias_grad_column_sum(dtype, rows, N):
    C = _C()
    torch.manual_seed(0)
    dy = torch.randn(rows, N, device="cuda").to(dtype)
    ref = dy.float().sum(0)
    out = C.bias_grad(dy)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out, ref, atol=1e-3 * math.sqrt(rows), rtol=1e-4)
    acc = torch.randn(N, device="cuda").to(dtype)
    want = (acc.float() + ref).to(dtype)
    assert C.bias_grad(dy, acc) is None
    torch.testing.assert_close(acc.float(), want.float(), atol=1e-3 * math.sqrt(rows) + (0.02 if dtype == torch.bfloat16 else 0), rtol=1e-2)


@pytest.mark.parametrize("acc_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("splits,shape", [(4, (1024, 1024)), (1, (8,)), (3, (3072, 1024)), (4, (24, 40))])
def test_splitk_accumulate(acc_dtype, splits, shape):
    """acc += part.sum(0) in one kernel (fp32 slice sum, then the bf16/fp32 accumulate)."""
    C = _C()
    torch.manual_seed(0)
    part = torch.randn(splits, *shape, device="cuda")
    acc = torch.randn(*shape, device="cuda").to(acc_dtype)
    want = (acc.float() + part.sum(0)).to(acc_dtype)
    C.splitk_accumulate(part, acc)
    torch.testing.assert_close(acc, want, atol=1e-5 if acc_dtype == torch.float32 else 0.05, rtol=1e-5 if acc_dtype == torch.float32 else 1e-2)
    C.splitk_accumulate(part, acc, accumulate=False)
    torch.testing.assert_close(acc.float(), part.sum(0).to(acc_dtype).float(), atol=1e-5 if acc_dtype == torch.float32 else 0.05, rtol=1e-2)
    with pytest.raises(RuntimeError):
        C.splitk_accumulate(part[:, :1], acc)


def _flat(params):
    from determined_clone_amd.parallel.flat import FlatParamSpace

    space = FlatParamSpace([params])
    calls = []
    for p in params:
        p.register_post_accumulate_grad_hook(lambda q, calls=calls: calls.append(id(q)))
    return space, calls


@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("seq", [96, 2048])
def test_linear_direct_grad_accumulation(bias, seq):
    """T.linear accumulates dW (GEMM beta=1, or 4-way split-K batched GEMM at >= 8k tokens) and db
    (fused column sum) into flat .grad views; equals autograd's F.linear over two backward
    passes; post-accumulate hooks fire."""
    _C()
    torch.manual_seed(0)
    from determined_clone_amd.ops import transformer as tr

    assert tr._wgrad_splits(4 * seq, 512, 256) == (4 if seq == 2048 else 1)
    x = torch.randn(4, seq, 256, device="cuda").bfloat16()
    g = torch.randn(4, seq, 512, device="cuda").bfloat16()
    w1 = torch.nn.Parameter(torch.randn(512, 256, device="cuda").bfloat16() * 0.05)
    b1 = torch.nn.Parameter(torch.randn(512, device="cuda").bfloat16()) if bias else None
    w2 = torch.nn.Parameter(w1.detach().clone())
    b2 = torch.nn.Parameter(b1.detach().clone()) if bias else None
    params = [p for p in (w1, b1) if p is not None]
    space, calls = _flat(params)
    ptrs = [p.grad.data_ptr() for p in params]
    xs = [x.clone().requires_grad_(True) for _ in range(2)]
    for _ in range(2):
        (T.linear(xs[0], w1, b1) * g).float().sum().backward()
        (torch.nn.functional.linear(xs[1], w2, b2) * g).float().sum().backward()
    from determined_clone_amd.ops import _grad

    _grad.join()  # weight and bias gradients accumulate on the side stream
    assert [p.grad.data_ptr() for p in params] == ptrs
    assert len(calls) == 2 * len(params)
    assert _rel(w1.grad, w2.grad) < 1e-2
    if bias:
        assert _rel(b1.grad, b2.grad) < 1e-2
    assert _rel(xs[0].grad, xs[1].grad) < 1e-2


def test_layer_norm_and_bias_gelu_direct_grad_accumulation():
    _C()
    torch.manual_seed(0)
    D, N = 256, 1024
    x = torch.randn(8, 64, D, device="cuda").bfloat16()
    r = torch.randn(8, 64, D, device="cuda").bfloat16()
    h = torch.randn(8, 64, N, device="cuda").bfloat16()
    lw1 = torch.nn.Parameter(torch.rand(D, device="cuda") + 0.5)
    lb1 = torch.nn.Parameter(torch.randn(D, device="cuda"))
    gb1 = torch.nn.Parameter(torch.randn(N, device="cuda").bfloat16())
    lw2, lb2, gb2 = (torch.nn.Parameter(p.detach().clone()) for p in (lw1, lb1, gb1))
    space, calls = _flat([lw1, lb1, gb1])
    for _ in range(2):
        for lw, lb, gb in ((lw1, lb1, gb1), (lw2, lb2, gb2)):
            y, s = T.layer_norm(x, lw, lb, 1e-5, residual=r)
            z = T.bias_gelu(h, gb)
            (y.float().square().sum() + s.float().sum() + z.float().sum()).backward()
    assert len(calls) == 6
    assert _rel(lw1.grad, lw2.grad) < 1e-4
    assert _rel(lb1.grad, lb2.grad) < 1e-4
    assert _rel(gb1.grad, gb2.grad) < 1e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("acc_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,D", [(333, 64), (8192, 768), (4096, 2048), (1024, 4096)])
def test_ln_bwd_dx_column_sums(dtype, acc_dtype, rows, D):
    """ln_bwd(colsum_acc=...) adds dx.sum(rows) into the target in the same pass (D <= 2048; a
    separate column reduction past that) and leaves dx / dgamma / dbeta unchanged."""
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(rows, D, device="cuda").to(dtype)
    dy = torch.randn(rows, D, device="cuda").to(dtype)
    ds = torch.randn(rows, D, device="cuda").to(dtype)
    w = torch.rand(D, device="cuda") + 0.5
    b = torch.randn(D, device="cuda")
    _, _, mean, rstd = C.ln_fwd(x, None, w, b, 1e-5, False)
    dx0, dg0, db0 = C.ln_bwd(dy, x, w, mean, rstd, ds, True)
    acc = torch.randn(D, device="cuda").to(acc_dtype)
    want = acc.float() + dx0.float().sum(0)
    dx1, dg1, db1 = C.ln_bwd(dy, x, w, mean, rstd, ds, True, None, None, acc)
    # same math; the two instantiations may contract multiply-adds differently (an ulp)
    ulp = 1e-5 if dtype == torch.float32 else 2 ** -7
    torch.testing.assert_close(dx1, dx0, atol=ulp * 4, rtol=ulp)
    torch.testing.assert_close(dg1, dg0, atol=1e-4 * math.sqrt(rows), rtol=1e-5)
    torch.testing.assert_close(db1, db0, atol=1e-4 * math.sqrt(rows), rtol=1e-5)
    # the kernel sums dx before its bf16 rounding: allow that rounding's random walk
    tol = 1e-3 * math.sqrt(rows) + (0.05 if acc_dtype == torch.bfloat16 else 0)
    if dtype == torch.bfloat16:
        tol += 2 ** -8 * math.sqrt(rows) * dx0.float().abs().max().item()
    torch.testing.assert_close(acc.float(), want, atol=tol, rtol=1e-2)


@pytest.mark.parametrize("extra_consumer", [False, True])
def test_out_projection_bias_grad_reduced_in_layer_norm_backward(extra_consumer, monkeypatch):
    """Pre-LN block pattern ``LN(resid + linear(h))``: the linear's bias gradient comes out of the
    LayerNorm backward (no separate column sum) and equals the unfused path's -- also when the
    linear output has a second consumer (only that consumer's share is reduced separately)."""
    _C()
    torch.manual_seed(0)
    D, N = 768, 1024
    h = torch.randn(4, 256, N, device="cuda").bfloat16()
    resid = torch.randn(4, 256, D, device="cuda").bfloat16()
    g = torch.randn(4, 256, D, device="cuda").bfloat16()
    w = torch.randn(D, N, device="cuda").bfloat16() * 0.03
    bias = torch.randn(D, device="cuda").bfloat16()
    lw = torch.rand(D, device="cuda") + 0.5
    lb = torch.randn(D, device="cuda")
    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(T, "FUSE_LN_BIAS_GRAD", fused)
        ps = [torch.nn.Parameter(t.clone()) for t in (w, bias, lw, lb)]
        space, _ = _flat(ps)
        hits = T.LN_BIAS_GRAD_HITS[0]
        for _ in range(2):
            out = T.linear(h, ps[0], ps[1])
            y, s = T.layer_norm(resid, ps[2], ps[3], 1e-5, residual=out)
            loss = (y.float() * g.float()).sum() + s.float().square().mean()
            if extra_consumer:
                loss = loss + (out.float() * 0.5).sum()
            loss.backward()
        from determined_clone_amd.ops import _grad

        _grad.join()
        assert T.LN_BIAS_GRAD_HITS[0] - hits == (2 if fused else 0)
        grads[fused] = [p.grad.float().clone() for p in ps]
    for a, b in zip(grads[True], grads[False]):
        assert _rel(a, b) < 2e-2


def test_hipblaslt_epilogue_probe_runs():
    """tools/lt_probe.py's entry point: the plain GEMM and the BIAS epilogue have kernels."""
    C = _C()
    torch.zeros(1, device="cuda")
    assert C.lt_probe(1, 1024, 4096, 1024, True, False, -1, -1, False) > 0
    assert C.lt_probe(4, 1024, 4096, 1024, True, False, 0, -1, True) > 0

