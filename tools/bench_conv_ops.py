"""Per-operation timing of ResNet-50's 1x1 convolutions (bs256, NHWC bf16): MIOpen (forward,
backward-data, backward-weight as separate aten.convolution_backward calls, each with whatever
memsets MIOpen issues) against hipBLASLt GEMMs on the [N*H*W, C] view (torch.mm; weight gradient
by addmm into a persistent bf16 .grad, beta=1, as the framework's flat-buffer accumulation would).

Decides, per shape and direction, which library runs the pointwise convolutions.
Usage: ``python tools/bench_conv_ops.py``; prints one JSON line per shape and per-step totals.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from determined_clone_amd.ops import miopen_db  # noqa: E402

miopen_db.use_private_copy("tools")  # never write the shipped DB from a bench

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (H_in, Cin, Cout, stride, count per ResNet-50 step)
SHAPES = [
    (56, 64, 64, 1, 1), (56, 256, 64, 1, 2), (56, 64, 256, 1, 4),      # layer1 (+ stride-1 ds)
    (56, 256, 128, 1, 1), (28, 512, 128, 1, 3), (28, 128, 512, 1, 4), (56, 256, 512, 2, 1),
    (28, 512, 256, 1, 1), (14, 1024, 256, 1, 5), (14, 256, 1024, 1, 6), (28, 512, 1024, 2, 1),
    (14, 1024, 512, 1, 1), (7, 2048, 512, 1, 2), (7, 512, 2048, 1, 3), (14, 1024, 2048, 2, 1),
]


def timed(fn, it=20):
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
    torch.backends.cudnn.benchmark = True
    N = 256
    tot = {}
    for H, ci, co, st, cnt in SHAPES:
        x = torch.randn(N, ci, H, H, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 1, 1, device="cuda") * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        Ho = (H - 1) // st + 1
        dy = torch.randn(N, co, Ho, Ho, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        bwd = torch.ops.aten.convolution_backward
        args = (dy, x, w, None, [st, st], [0, 0], [1, 1], False, [0, 0], 1)
        r = {"H": H, "cin": ci, "cout": co, "stride": st, "count": cnt}
        r["mi_fwd"] = timed(lambda: F.conv2d(x, w, stride=st))
        r["mi_dgrad"] = timed(lambda: bwd(*args, [True, False, False]))
        r["mi_wgrad"] = timed(lambda: bwd(*args, [False, True, False]))
        # GEMM forms on the NHWC [rows, C] view (stride 2: strided input view copied first)
        X = x.permute(0, 2, 3, 1)
        if st != 1:
            X = X[:, ::st, ::st, :]
        W = w.view(co, ci)
        DY = dy.permute(0, 2, 3, 1).reshape(-1, co)
        g = torch.zeros(co, ci, device="cuda", dtype=torch.bfloat16)
        r["mm_fwd"] = timed(lambda: torch.mm(X.reshape(-1, ci), W.t()))
        if st == 1:
            r["mm_dgrad"] = timed(lambda: torch.mm(DY, W))
        X2 = X.reshape(-1, ci)
        r["mm_wgrad_acc_bf16"] = timed(lambda: g.addmm_(DY.t(), X2))
        r["mm_wgrad"] = timed(lambda: torch.mm(DY.t(), X2))
        for k, v in r.items():
            if isinstance(v, float):
                r[k] = round(v, 1)
                tot[k] = tot.get(k, 0.0) + v * cnt
        print(json.dumps(r), flush=True)
    print(json.dumps({"per_step_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
