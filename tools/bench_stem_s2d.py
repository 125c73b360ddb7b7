"""Time the stem space-to-depth (csrc/conv_igemm.hip stem_s2d) against ATen's pad + reshape on the
ResNet-50 bs-1024 image batch: python tools/bench_stem_s2d.py [--batch 1024]."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from determined_clone_amd.ops import _ext  # noqa: E402


def _aten(x):
    n, c, h, w = x.shape
    xn = F.pad(x.permute(0, 2, 3, 1), (0, 0, 3, 3, 3, 3)).view(n, (h + 6) // 2, 2, (w + 6) // 2, 2, c)
    return xn.permute(0, 1, 3, 2, 4, 5).reshape(n, (h + 6) // 2, (w + 6) // 2, 4 * c)


def _time(fn, x, iters=20):
    for _ in range(3):
        fn(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn(x)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    x = torch.randn(args.batch, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    C = _ext.load()
    nbytes = x.numel() * 2 + args.batch * 12 * 115 * 115 * 2
    for name, fn in (("hip stem_s2d", C.stem_s2d), ("aten pad+reshape", _aten)):
        us = _time(fn, x)
        print(f"{name:18s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s (read image + write s2d)")


if __name__ == "__main__":
    main()
