"""MIOpen exhaustive tuning of the ResNet-50 weight gradients at batch 1024 (the side stream's
MIOpen backward-weight problems). ``time SET`` prints immediate-mode times with the DB in
MIOPEN_USER_DB_PATH; ``tune SET`` runs MIOpen find with MIOPEN_FIND_ENFORCE=SEARCH (set by the
caller) on each problem so the perf DB there records tuned parameters. SET: 3x3 or 1x1."""
import json
import sys
import time

import torch

SHAPES3 = [(56, 64, 64, 1), (56, 128, 128, 2), (28, 128, 128, 1), (28, 256, 256, 2),
           (14, 256, 256, 1), (14, 512, 512, 2), (7, 512, 512, 1)]
SHAPES1 = [(56, 64, 64, 1), (56, 256, 64, 1), (56, 64, 256, 1), (56, 256, 128, 1),
           (56, 256, 512, 2), (28, 512, 128, 1), (28, 128, 512, 1), (28, 512, 256, 1),
           (28, 512, 1024, 2), (14, 1024, 256, 1), (14, 256, 1024, 1), (14, 1024, 512, 1),
           (14, 1024, 2048, 2), (7, 2048, 512, 1), (7, 512, 2048, 1)]


def timed(fn, iters=8):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    mode, which = sys.argv[1], sys.argv[2]
    torch.backends.cudnn.benchmark = mode == "tune"
    k = 3 if which == "3x3" else 1
    cl = torch.channels_last
    for H, ci, co, st in (SHAPES3 if k == 3 else SHAPES1):
        pad = 1 if k == 3 else 0
        x = torch.randn(1024, ci, H, H, device="cuda").bfloat16().contiguous(memory_format=cl)
        w = (torch.randn(co, ci, k, k, device="cuda") * 0.05).bfloat16().contiguous(memory_format=cl)
        ho = (H + 2 * pad - k) // st + 1
        dy = torch.randn(1024, co, ho, ho, device="cuda").bfloat16().contiguous(memory_format=cl)
        fn = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
            dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1, [False, True, False])
        t = time.perf_counter()
        if mode == "tune":
            fn()
            torch.cuda.synchronize()
            print(json.dumps({"shape": [H, ci, co, st, k], "tune_s": round(time.perf_counter() - t, 1)}), flush=True)
        else:
            print(json.dumps({"shape": [H, ci, co, st, k], "wgrad_us": round(timed(fn), 1)}), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
