"""Microbenchmark: fused NHWC BatchNorm(+ReLU) train forward + backward on every distinct ResNet-50
BN shape at batch 256 (bf16), reporting achieved HBM bandwidth per shape and the step-weighted
total (each shape weighted by how often it occurs in ResNet-50).

Usage: ``python tools/bench_bn.py [--batch 256]``; set ``DCA_BN_REDUCE=elems,min,max`` to try a
different reduce-grid heuristic. Small shapes are launch/CPU bound in this eager loop (fwd + bwd
= 6 kernels + autograd): read per-kernel times from ``rocprofv3 --kernel-trace`` for those.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from determined_clone_amd.ops import batchnorm as bn  # noqa: E402

# (C, H*W, count in ResNet-50); stem excluded (fused with maxpool).
SHAPES = [(64, 56 * 56, 6), (256, 56 * 56, 4), (128, 56 * 56, 1), (128, 28 * 28, 7),
          (512, 28 * 28, 5), (256, 28 * 28, 1), (256, 14 * 14, 11), (1024, 14 * 14, 7),
          (512, 14 * 14, 1), (512, 7 * 7, 5), (2048, 7 * 7, 4)]


def timed(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda")
    tot_f = tot_b = 0.0
    print(f"DCA_BN_REDUCE={os.environ.get('DCA_BN_REDUCE', 'default')}")
    print(f"{'C':>5} {'HW':>5} {'n':>2} {'MB':>7} {'fwd us':>8} {'fwd TB/s':>8} {'bwd us':>8} {'bwd TB/s':>8}")
    for C, HW, n in SHAPES:
        x = torch.randn(args.batch, C, HW // int(HW ** 0.5), int(HW ** 0.5), device=dev,
                        dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w = torch.ones(C, device=dev, requires_grad=True)
        b = torch.zeros(C, device=dev, requires_grad=True)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y = bn.batch_norm_act(x, w, b, rm, rv)
        g = torch.randn_like(y)
        mb = x.numel() * 2 / 1e6
        tf = timed(lambda: bn.batch_norm_act(x, w, b, rm, rv))

        def fb():
            out = bn.batch_norm_act(x, w, b, rm, rv)
            torch.autograd.grad(out, (x, w, b), g)

        tfb = timed(fb)
        tb = tfb - tf
        # fwd: read x twice + write y; bwd: read dy, x twice each + write dx (+ mask bits)
        print(f"{C:5d} {HW:5d} {n:2d} {mb:7.1f} {tf:8.1f} {3 * mb / tf:8.2f} {tb:8.1f} "
              f"{5 * mb / tb:8.2f}")
        tot_f += n * tf
        tot_b += n * tb
    print(f"weighted per-step: fwd {tot_f / 1e3:.3f} ms, bwd {tot_b / 1e3:.3f} ms, "
          f"total {(tot_f + tot_b) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
