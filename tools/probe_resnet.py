"""Quick ResNet-50 training-step probe (no harness): torch BN vs fused HIP BN, bf16 NHWC."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from determined_clone_amd.models import resnet
from determined_clone_amd.ops import batchnorm, optim as fopt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bn", default="fused", choices=["fused", "torch"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--opt", default="fused", choices=["fused", "torch"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "amp"])
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    if args.bn == "torch":
        orig = batchnorm.batch_norm_act

        def torch_bn(x, w, b, rm, rv, residual=None, training=True, momentum=0.1, eps=1e-5,
                     relu=True, num_batches_tracked=None):
            return batchnorm.reference_batch_norm_act(x, w, b, rm, rv, residual, training,
                                                      momentum, eps, relu)

        resnet.bn_ops.batch_norm_act = torch_bn
    dev = torch.device("cuda")
    model = resnet.resnet50().to(dev)
    if args.dtype == "bf16":
        model = resnet.to_mi355x_layout(model)
    else:
        model = model.to(memory_format=torch.channels_last)
    if args.opt == "fused":
        opt = fopt.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    B = args.batch
    x = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)

    def step():
        opt.zero_grad()
        if args.dtype == "amp":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x)
        else:
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    t0 = time.time()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t1 = time.time()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    t2 = time.time()
    ms = (t2 - t1) / args.steps * 1000
    print(json.dumps({"bn": args.bn, "opt": args.opt, "dtype": args.dtype, "batch": B,
                      "warmup_s": round(t1 - t0, 2), "ms_per_step": round(ms, 2),
                      "img_per_s": round(B / ms * 1000, 1), "loss": float(loss),
                      "mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
