"""Latent-diffusion family on MI355X: bf16 NHWC UNet / VAE / text encoder with the MFMA
flash-attention kernels vs the fp32 CPU oracle of the same weights; textual inversion steps with
the fused HIP Adam."""
import pytest
import torch

from determined_clone_amd.models import diffusion as ldm
from determined_clone_amd.model_hub.diffusion import TextualInversionTrainer

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def test_unet_vae_text_bf16_match_fp32():
    torch.manual_seed(0)
    cpu = ldm.LatentDiffusion(ldm.LDMConfig.preset("tiny")).eval()
    torch.manual_seed(0)
    gpu = ldm.LatentDiffusion(ldm.LDMConfig.preset("tiny")).eval().to_mi355x_layout(torch.device("cuda"))
    x = torch.randn(2, 3, 64, 64)
    ids = cpu.tokenizer(["a photo of a cat", "a dog"])
    t = torch.tensor([5, 700])
    with torch.no_grad():
        ctx_c = cpu.text_encoder(ids)
        ctx_g = gpu.text_encoder(ids.cuda())
        assert _rel(ctx_g.cpu(), ctx_c) < 3e-2
        mean_c, _ = cpu.vae.encode(x)
        xg = x.cuda().bfloat16().contiguous(memory_format=torch.channels_last)
        mean_g, _ = gpu.vae.encode(xg)
        assert _rel(mean_g.cpu(), mean_c) < 5e-2
        z = mean_c
        eps_c = cpu.unet(z, t, ctx_c)
        zg = z.cuda().bfloat16().contiguous(memory_format=torch.channels_last)
        eps_g = gpu.unet(zg, t.cuda(), ctx_c.cuda().bfloat16())
        assert _rel(eps_g.cpu(), eps_c) < 5e-2


def test_unet_backward_through_flash_attention():
    torch.manual_seed(0)
    m = ldm.LatentDiffusion(ldm.LDMConfig.preset("tiny")).to_mi355x_layout(torch.device("cuda"))
    z = torch.randn(2, 4, 8, 8, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ctx = m.encode_text(["a", "b"]).detach().requires_grad_(True)
    out = m.unet(z, torch.tensor([1, 2], device="cuda"), ctx)
    out.float().square().mean().backward()
    assert ctx.grad is not None and torch.isfinite(ctx.grad).all() and ctx.grad.abs().sum() > 0
    assert all(torch.isfinite(p.grad).all() for p in m.unet.parameters() if p.grad is not None)


def test_textual_inversion_steps_on_gpu():
    tr = TextualInversionTrainer(["det-logo"], ["brain logo"], ["object"], ["/nonexistent"],
                                 model_preset="tiny", img_size=64, train_batch_size=2,
                                 learning_rate=1e-2)
    assert tr.device.type == "cuda"
    before = tr.new_embedding.weight.detach().clone()
    base = tr.model.text_encoder.token_embedding.original.weight.detach().clone()
    tr.train_steps(2)
    torch.cuda.synchronize()
    assert tr.new_embedding.weight.dtype == torch.float32
    assert not torch.equal(before, tr.new_embedding.weight)
    assert torch.equal(base, tr.model.text_encoder.token_embedding.original.weight)
    imgs = tr.generate(["a det-logo"], seed=1)
    assert imgs.shape == (1, 64, 64, 3)


def test_unet_flat_grads_side_stream_match_autograd():
    """Fused linear / LayerNorm / GroupNorm / conv paths accumulating into flat .grad views
    (side-stream weight gradients included) give the same gradients as plain autograd."""
    import copy

    from determined_clone_amd.ops import _grad
    from determined_clone_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    ref = ldm.to_mi355x_layout(ldm.UNet2DCondition(ldm.UNetConfig.tiny()), torch.device("cuda"))
    m = copy.deepcopy(ref)
    FlatParamSpace([[p for p in m.parameters() if p.dtype == torch.bfloat16],
                    [p for p in m.parameters() if p.dtype == torch.float32]])
    z = torch.randn(2, 4, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    ctx = torch.randn(2, 16, 64, device="cuda").bfloat16()
    t = torch.tensor([3, 600], device="cuda")
    m(z, t, ctx).float().square().mean().backward()
    _grad.join()
    ref(z, t, ctx).float().square().mean().backward()
    for (n, a), b in zip(m.named_parameters(), ref.parameters()):
        ga, gb = a.grad.float(), b.grad.float()
        assert (ga - gb).norm() <= 3e-2 * gb.norm() + 1e-4, n
