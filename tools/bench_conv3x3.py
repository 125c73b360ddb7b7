"""Per-direction timing of ResNet-50's 3x3 convolutions and the 7x7 stem through MIOpen (NHWC bf16,
immediate mode from the shipped find DB, as bench.py runs them) at the bench batch: achieved
TFLOP/s and HBM GB/s per shape, and per-step totals. Usage: ``python tools/bench_conv3x3.py
[--batch 1024]``."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from determined_clone_amd.ops import miopen_db  # noqa: E402

miopen_db.use_private_copy("tools")  # never write the shipped DB from a bench

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (H_in, Cin, Cout, k, stride, pad, count per ResNet-50 step)
SHAPES = [
    (224, 3, 64, 7, 2, 3, 1),
    # stem variants with the same math: input channels zero-padded to 4 / 8, and space-to-depth
    # (7x7/2 on 230x230x3 == 4x4/1 on 115x115x12 with a re-packed weight)
    (224, 4, 64, 7, 2, 3, 0), (224, 8, 64, 7, 2, 3, 0), (115, 12, 64, 4, 1, 0, 0),
    (56, 64, 64, 3, 1, 1, 3),
    (56, 128, 128, 3, 2, 1, 1), (28, 128, 128, 3, 1, 1, 3),
    (28, 256, 256, 3, 2, 1, 1), (14, 256, 256, 3, 1, 1, 5),
    (14, 512, 512, 3, 2, 1, 1), (7, 512, 512, 3, 1, 1, 2),
]


def timed(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3  # us


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--find", action="store_true", help="MIOpen find (cudnn.benchmark) instead of "
                    "immediate mode: needed for shapes the shipped find DB does not hold")
    ap.add_argument("--only-stem", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.find
    n = a.batch
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for H, ci, co, k, st, pad, cnt in SHAPES:
        if a.only_stem and H < 100:
            continue
        x = torch.randn(n, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, k, k, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=st, padding=pad)
        g = torch.randn_like(y)
        Ho = y.shape[2]
        flops = 2.0 * n * Ho * Ho * co * ci * k * k
        fwd = timed(lambda: F.conv2d(x, w, stride=st, padding=pad))
        res = {"H": H, "cin": ci, "cout": co, "k": k, "stride": st, "count": cnt,
               "fwd_us": round(fwd, 1), "fwd_tflops": round(flops / fwd / 1e6, 1)}
        dirs = [("wgrad", (False, True, False))]
        if ci > 3:
            dirs.insert(0, ("dgrad", (True, False, False)))
        for name, mask in dirs:
            t = timed(lambda: torch.ops.aten.convolution_backward(
                g, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, list(mask)))
            res[f"{name}_us"] = round(t, 1)
            res[f"{name}_tflops"] = round(flops / t / 1e6, 1)
            tot[name] += t * cnt
        tot["fwd"] += fwd * cnt
        bytes_io = (x.numel() + y.numel()) * 2
        res["io_roof_us"] = round(bytes_io / 5.0e6, 1)  # in + out at 5 TB/s
        print(json.dumps(res), flush=True)
        del x, w, y, g
        torch.cuda.empty_cache()
    print(json.dumps({"per_step_ms": {k_: round(v / 1e3, 2) for k_, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
