"""MIOpen exhaustive tuning of the ResNet-50 stem (the 12-channel 4x4/1 space-to-depth convolution at
batch 1024): ``time`` reports the immediate-mode forward / weight-gradient times with the DB in
MIOPEN_USER_DB_PATH; ``tune`` runs MIOpen find with MIOPEN_FIND_ENFORCE=SEARCH (set by the caller)
so the perf DB there records tuned parameters for these two problems."""
import json
import sys
import time

import torch
import torch.nn.functional as F


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    mode = sys.argv[1]
    torch.backends.cudnn.benchmark = mode == "tune"
    cl = torch.channels_last
    xs = torch.randn(1024, 12, 115, 115, device="cuda").bfloat16().contiguous(memory_format=cl)
    w2 = (torch.randn(64, 12, 4, 4, device="cuda") * 0.1).bfloat16().contiguous(memory_format=cl)
    dy = torch.randn(1024, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=cl)
    fwd = lambda: F.conv2d(xs, w2)  # noqa: E731
    wgr = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
        dy, xs, w2, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])
    if mode == "tune":
        for name, fn in (("fwd", fwd), ("wgrad", wgr)):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            print(json.dumps({"tuned": name, "s": round(time.perf_counter() - t, 1)}), flush=True)
        return
    print(json.dumps({"fwd_us": round(timed(fwd), 1), "wgrad_us": round(timed(wgr), 1)}), flush=True)


if __name__ == "__main__":
    main()
