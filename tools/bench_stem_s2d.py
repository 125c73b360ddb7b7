"""Time the ResNet-50 stem pieces on the bs-1024 image batch: the space-to-depth
(csrc/conv_igemm.hip stem_s2d) against ATen's pad + reshape, and the stem convolution kernel
(stem_conv_kernel, BatchNorm statistics included) against MIOpen's S2D convolution plus the separate
statistics pass: python tools/bench_stem_s2d.py [--batch 1024]."""
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
    from determined_clone_amd.ops import conv

    torch.manual_seed(0)
    w = torch.randn(64, 3, 7, 7, device="cuda").bfloat16()
    xs16, w16 = C.stem_s2d(x, 16), conv._s2d_weight(w, 16)
    xs12, w12 = C.stem_s2d(x, 12), conv._s2d_weight(w)
    y = C.stem_conv_fwd(xs16, w16)[0]
    flops = 2.0 * y.numel() * 147
    ybytes = y.numel() * 2

    for name, fn, arg in (("hip stem_conv+stats", lambda a: C.stem_conv_fwd(a, w16), xs16),
                          ("miopen conv only", lambda a: F.conv2d(a, w12), xs12)):
        us = _time(fn, arg)
        print(f"{name:20s} {us:8.1f} us  {flops / us / 1e6:7.1f} TFLOP/s (7x7 flops)  "
              f"{(ybytes + arg.numel() * 2) / us / 1e6:5.2f} TB/s")
    # the weight gradient (MIOpen, on the side stream in the step; the last kernel of backward)
    dy = torch.randn_like(y)
    for name, xs, w2 in (("miopen wgrad C=16", xs16, w16), ("miopen wgrad C=12", xs12, w12)):
        args = (dy, xs, w2, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])
        us = _time(lambda a: torch.ops.aten.convolution_backward(*a), args)
        print(f"{name:20s} {us:8.1f} us")
    us = _time(lambda a: C.stem_wgrad(*a), (dy, xs12))
    print(f"{'hip stem_wgrad':20s} {us:8.1f} us  {2.0 * y.numel() * 192 / us / 1e6:7.1f} TFLOP/s (S2D flops)  "
          f"{(y.numel() + xs12.numel()) * 2 / us / 1e6:5.2f} TB/s")


if __name__ == "__main__":
    main()
