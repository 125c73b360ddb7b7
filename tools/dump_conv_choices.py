"""Measure the ops/conv.py chooser decisions on this GPU and write them to
``ops/tuned/conv_choices_gfx950.json`` (shipped, so bench / trial processes never time them).

The headline shapes are best recorded from the real bench process, whose step conditions
(flat .grad views, side-stream weight gradients) the timings depend on:
``DCA_CONV_CHOICES=0 DCA_CONV_DUMP=<file> python bench.py`` (ops/conv.py dumps its decisions at
exit, merging into the file). This tool adds the remaining workloads to the same file -- ResNet-50
at bs 256 and the SD-2-shaped UNet at bs 8 / 512^2 -- with the shipped file ignored. GPU only.

Usage: python tools/dump_conv_choices.py [--out PATH] [--batches 256] [--skip-unet]
"""
import argparse
import os
import sys

os.environ["DCA_CONV_CHOICES"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--skip-unet", action="store_true")
    ap.add_argument("--batches", default="1024,256", help="ResNet-50 batch sizes to run")
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F

    from determined_clone_amd.models import resnet
    from determined_clone_amd.ops import conv as conv_ops
    from determined_clone_amd.ops import optim as fopt

    dev = torch.device("cuda")
    out = a.out or conv_ops._SHIPPED_PATH
    if os.path.exists(out):  # keep decisions already recorded (e.g. by the bench process)
        conv_ops.load_choices(out)
    for bs in [int(b) for b in a.batches.split(",") if b]:
        torch.manual_seed(0)
        model = resnet.to_mi355x_layout(resnet.resnet50()).to(dev)
        opt = fopt.FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
        x = torch.randn(bs, 3, 224, 224, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (bs,), device=dev)
        for _ in range(2):
            F.cross_entropy(model(x).float(), y).backward()
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        print(f"resnet50 bs {bs}: {len(conv_ops._CHOICE)} decisions so far", flush=True)
        del model, opt, x
        torch.cuda.empty_cache()
    if not a.skip_unet:
        from determined_clone_amd.models import diffusion as ldm

        cfg = ldm.LDMConfig.preset("sd2-base")
        unet = ldm.to_mi355x_layout(ldm.UNet2DCondition(cfg.unet), dev)
        opt = fopt.FusedAdamW(unet.parameters(), lr=1e-5)
        z = torch.randn(8, 4, 64, 64, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        ctx = torch.randn(8, cfg.text.max_length, cfg.unet.cross_attention_dim, device=dev).bfloat16()
        t = torch.randint(0, 1000, (8,), device=dev)
        for _ in range(2):
            F.mse_loss(unet(z, t, ctx).float(), torch.zeros_like(z, dtype=torch.float32)).backward()
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        print(f"unet: {len(conv_ops._CHOICE)} decisions so far", flush=True)
    conv_ops.dump_choices(out, torch.cuda.get_device_name(0))
    print(f"wrote {len(conv_ops._CHOICE)} decisions ({conv_ops.TIMINGS} candidate timings) to {out}")


if __name__ == "__main__":
    main()
