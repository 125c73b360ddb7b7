"""Micro-benchmarks of the transformer backward's memory-bound kernels at GPT-2-medium micro-32
shapes (32768 tokens, d_model 1024): LayerNorm backward (+ residual gradient, + affine
accumulation), the bias-gradient column sum, and the split-K weight-gradient epilogue (fused
``splitk_accumulate`` vs the previous torch ``sum(0)`` + ``add_``). One JSON line per case with
achieved HBM GB/s (bytes each kernel must move)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402
from determined_clone_amd.ops import transformer as T  # noqa: E402


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


def main():
    C = _ext.load()
    rows, E = 32768, 1024
    out = []
    x = torch.randn(rows, E, device="cuda").bfloat16().requires_grad_(True)
    r = torch.randn(rows, E, device="cuda").bfloat16().requires_grad_(True)
    w = torch.ones(E, device="cuda", requires_grad=True)
    b = torch.zeros(E, device="cuda", requires_grad=True)
    y, s = T.layer_norm(x, w, b, 1e-5, residual=r)
    gy, gs = torch.randn_like(y), torch.randn_like(s)
    ms = timeit(lambda: torch.autograd.grad((y, s), (x, r, w, b), (gy, gs), retain_graph=True))
    # dy, dsum, sum (x) read; dx written (dres aliases dx: autograd returns it for both inputs)
    out.append({"op": "ln_bwd+dres", "blocks": os.environ.get("DCA_LN_BWD_BLOCKS", "default"),
                "ms": ms, "GBps": 4 * rows * E * 2 / ms / 1e6})
    for N in (1024, 3072, 4096):
        dy = torch.randn(rows, N, device="cuda").bfloat16()
        acc = torch.zeros(N, device="cuda").bfloat16()
        ms = timeit(lambda: C.bias_grad(dy, acc))
        out.append({"op": "bias_grad", "N": N, "ms": ms, "GBps": rows * N * 2 / ms / 1e6})
    for m, n in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        dy2 = torch.randn(rows, m, device="cuda").bfloat16()
        x2 = torch.randn(rows, n, device="cuda").bfloat16()
        acc = torch.zeros(m, n, device="cuda").bfloat16()
        a = dy2.reshape(4, rows // 4, m).transpose(1, 2)
        bb = x2.reshape(4, rows // 4, n)

        def old():
            acc.add_(torch.bmm(a, bb).sum(0, dtype=torch.float32))

        def new():
            C.splitk_accumulate(torch.bmm(a, bb, out_dtype=torch.float32), acc)

        def gemm_only():
            torch.bmm(a, bb, out_dtype=torch.float32)

        def nosplit():
            acc.addmm_(dy2.t(), x2)

        t_old, t_new, t_g, t_ns = timeit(old), timeit(new), timeit(gemm_only), timeit(nosplit)
        out.append({"op": "wgrad_splitk", "m": m, "n": n, "old_ms": t_old, "new_ms": t_new,
                    "bmm_f32_ms": t_g, "addmm_nosplit_ms": t_ns,
                    "new_tflops": 2 * rows * m * n / t_new / 1e9})
    for o in out:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in o.items()}), flush=True)


if __name__ == "__main__":
    main()
