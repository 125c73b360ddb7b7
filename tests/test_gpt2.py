"""GPT-2 / NeoX model on the CPU reference path (+ one GPU bf16 parity test)."""
import pytest
import torch
import torch.nn.functional as F

from determined_clone_amd.models import gpt2


def _naive_forward(model: gpt2.GPT, idx: torch.Tensor) -> torch.Tensor:
    """Independent plain-PyTorch implementation of the same network (unfused residual adds,
    SDPA attention) used as the oracle."""
    cfg = model.cfg
    B, S = idx.shape
    x = model.wte(idx).float()
    if model.wpe is not None:
        x = x + model.wpe.weight[:S].float()
    for blk in model.blocks:
        h = F.layer_norm(x, (cfg.d_model,), blk.ln1.weight.float(), blk.ln1.bias.float(), cfg.ln_eps)
        qkv = F.linear(h, blk.attn.qkv.weight.float(), blk.attn.qkv.bias.float())
        q, k, v = qkv.view(B, S, 3, cfg.n_head, cfg.head_dim).unbind(2)
        if blk.attn.rot:
            from determined_clone_amd.ops import transformer as T

            q = T.reference_rope(q, model.rope_cos, model.rope_sin, blk.attn.rot)
            k = T.reference_rope(k, model.rope_cos, model.rope_sin, blk.attn.rot)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           is_causal=True).transpose(1, 2).reshape(B, S, -1)
        x = x + F.linear(o, blk.attn.proj.weight.float(), blk.attn.proj.bias.float())
        h = F.layer_norm(x, (cfg.d_model,), blk.ln2.weight.float(), blk.ln2.bias.float(), cfg.ln_eps)
        m = F.gelu(F.linear(h, blk.mlp.fc.weight.float(), blk.mlp.fc.bias.float()), approximate="tanh")
        x = x + F.linear(m, blk.mlp.proj.weight.float(), blk.mlp.proj.bias.float())
    x = F.layer_norm(x, (cfg.d_model,), model.ln_f.weight.float(), model.ln_f.bias.float(), cfg.ln_eps)
    return F.linear(x, model.wte.weight.float())


@pytest.mark.parametrize("pos", ["learned", "rotary"])
def test_gpt_matches_naive_and_is_causal(pos):
    torch.manual_seed(0)
    m = gpt2.gpt2("tiny", pos_emb=pos)
    idx = torch.randint(0, 512, (2, 33))
    logits, loss = m(idx, torch.randint(0, 512, (2, 33)))
    torch.testing.assert_close(logits, _naive_forward(m, idx), atol=1e-4, rtol=1e-4)
    assert abs(loss.item() - torch.log(torch.tensor(512.0)).item()) < 0.5
    idx2 = idx.clone()
    idx2[:, 20:] = torch.randint(0, 512, (2, 13))
    l2 = m(idx2)
    torch.testing.assert_close(l2[:, :20], logits[:, :20])
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


def test_gpt_trains_on_cpu():
    torch.manual_seed(0)
    m = gpt2.gpt2("tiny", n_layer=1)
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    idx = torch.randint(0, 512, (4, 32))
    first = None
    for _ in range(30):
        _, loss = m(idx, idx.roll(-1, 1))
        first = first or loss.item()
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert loss.item() < first * 0.5


def test_presets_and_flops():
    cfg = gpt2.config_for("gpt2-medium")
    assert (cfg.n_layer, cfg.d_model, cfg.head_dim, cfg.padded_vocab) == (24, 1024, 64, 50304)
    m = gpt2.gpt2("tiny")
    assert m.flops_per_token() > 6 * m.num_params()


def test_cast_keeps_layernorm_fp32():
    m = gpt2.cast_for_mi355x(gpt2.gpt2("tiny"))
    assert m.blocks[0].ln1.weight.dtype == torch.float32
    assert m.blocks[0].attn.qkv.weight.dtype == torch.bfloat16
    assert m.wte.weight.dtype == torch.bfloat16


@pytest.mark.gpu
@pytest.mark.parametrize("pos", ["learned", "rotary"])
def test_gpt_bf16_gpu_matches_fp32(pos):
    torch.manual_seed(0)
    m = gpt2.gpt2("tiny", pos_emb=pos, max_seq_len=256).cuda()
    idx = torch.randint(0, 512, (2, 200), device="cuda")
    ref = _naive_forward(m, idx)
    mb = gpt2.cast_for_mi355x(m)
    logits, loss = mb(idx, idx)
    rel = ((logits.float() - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    loss.backward()
    assert all(torch.isfinite(p.grad).all() for p in mb.parameters())
