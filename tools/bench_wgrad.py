"""Weight-gradient GEMM (dW += dY^T X, K = tokens) as one addmm_ vs split-K batched GEMM + sum,
at GPT-2-medium shapes (16k tokens). Prints ms per variant."""
import json

import torch


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def split_k(acc, dy, x, s):
    T, M = dy.shape
    N = x.shape[1]
    a = dy.view(s, T // s, M).transpose(1, 2)
    b = x.view(s, T // s, N)
    acc.add_(torch.bmm(a, b).sum(0, dtype=torch.float32).to(acc.dtype))


def main():
    T = 16384
    for M, N in ((1024, 1024), (3072, 1024), (4096, 1024), (1024, 4096)):
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        acc = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        res = {"M": M, "N": N, "K": T}
        base = timeit(lambda: acc.addmm_(dy.t(), x))
        res["addmm"] = round(base, 4)
        for s in (2, 4, 8):
            res[f"split{s}"] = round(timeit(lambda: split_k(acc, dy, x, s)), 4)
        fl = 2 * M * N * T
        res["addmm_tflops"] = round(fl / base / 1e9, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
