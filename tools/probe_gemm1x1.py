"""Probe: ResNet-50 1x1 convolutions (bs 256, NHWC bf16) as MIOpen convs vs plain GEMMs on the
channels_last storage ([N*H*W, Cin] x [Cin, Cout]), for forward, backward-data and weight-grad.
Prints time, TFLOP/s and the HBM-bound floor (bytes / 5 TB/s) per shape."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [(56, 64, 64, 3), (56, 256, 64, 2), (56, 64, 256, 4), (28, 128, 512, 4), (28, 512, 128, 3),
          (14, 256, 1024, 6), (14, 1024, 256, 5), (7, 512, 2048, 3), (7, 2048, 512, 2)]


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
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    N = 256
    tot = {"conv": 0.0, "gemm": 0.0, "floor": 0.0}
    for H, cin, cout, count in SHAPES:
        M = N * H * H
        x = torch.randn(N, cin, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, cout, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x2 = x.permute(0, 2, 3, 1).reshape(M, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(M, cout)
        w2 = w.view(cout, cin)
        res = {"H": H, "cin": cin, "cout": cout}
        flops = 2.0 * M * cin * cout
        for name, conv_fn, gemm_fn, nbytes in (
                ("fwd", lambda: F.conv2d(x, w), lambda: x2 @ w2.t(), 2 * M * (cin + cout)),
                ("dgrad", lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)),
                 lambda: dy2 @ w2, 2 * M * (cin + cout)),
                ("wgrad", lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)),
                 lambda: dy2.t() @ x2, 2 * M * (cin + cout))):
            tc, tg = timed(conv_fn), timed(gemm_fn)
            floor = nbytes / 5e12 * 1e3
            res[name] = {"conv_ms": round(tc, 4), "gemm_ms": round(tg, 4), "floor_ms": round(floor, 4),
                         "conv_tflops": round(flops / tc / 1e9, 1), "gemm_tflops": round(flops / tg / 1e9, 1)}
            tot["conv"] += count * tc
            tot["gemm"] += count * min(tg, tc)
            tot["floor"] += count * max(floor, flops / 2.0e15 * 1e3)
        print(json.dumps(res), flush=True)
    print(json.dumps({"per_step_ms": {k: round(v, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
