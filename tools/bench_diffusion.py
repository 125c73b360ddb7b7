"""Microbenchmark: SD2-base-shaped latent-diffusion UNet (865M params) training step on MI355X --
bf16 NHWC, MFMA flash attention, fused NHWC GroupNorm+SiLU, fused HIP AdamW over the UNet.
Prints one JSON line (``DCA_GN_TORCH=1`` runs GroupNorm through PyTorch for an A/B).

Usage: ``python tools/bench_diffusion.py [--batch 8 --res 512 --steps 10 --warmup 3]``.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DCA_GEMM_TUNED", "1")  # replay the shipped tuned GEMMs (ops/gemm_tuning.py)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from determined_clone_amd.models import diffusion as ldm  # noqa: E402
from determined_clone_amd.ops import optim as fopt  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", default="sd2-base")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    cfg = ldm.LDMConfig.preset(args.preset)
    torch.manual_seed(0)
    unet = ldm.to_mi355x_layout(ldm.UNet2DCondition(cfg.unet), dev)
    text = ldm.TextEncoder(cfg.text).to(dev, torch.bfloat16)
    opt = fopt.FusedAdamW(unet.parameters(), lr=1e-5)
    lat = args.res // 8
    z = torch.randn(args.batch, 4, lat, lat, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    noise = torch.randn_like(z, dtype=torch.float32)
    ids = torch.randint(0, cfg.text.vocab_size, (args.batch, cfg.text.max_length), device=dev)
    with torch.no_grad():
        ctx = text(ids)
    t = torch.randint(0, 1000, (args.batch,), device=dev)

    def step():
        pred = unet(z, t, ctx).float()
        F.mse_loss(pred, noise).backward()
        opt.step()
        opt.zero_grad()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    params = sum(p.numel() for p in unet.parameters())
    print(json.dumps({"mode": "unet_train_step", "preset": args.preset, "batch": args.batch,
                      "res": args.res, "ms_per_step": round(ms, 2),
                      "images_per_s": round(args.batch / ms * 1e3, 1), "unet_params_M": round(params / 1e6, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
