"""LayerNorm backward (and, with --bias-gelu, bias-GELU backward) micro-benchmark (``ln_bwd``: dx [+ residual gradient], dgamma / dbeta
accumulation, optional dx column sums = the out-projection bias gradient) at transformer widths.
Kernel path / shape knobs are read from the environment once per process (``DCA_LN_BWD_RG``,
``DCA_LN_BWD_ROWS``, ``DCA_LN_BWD_BLOCKS``), so a sweep runs one process per setting. One JSON
line per case with the achieved HBM GB/s over the bytes the pass must move."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=50, warmup=10):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    ap.add_argument("--widths", default="768,1024,1600,2048")
    ap.add_argument("--bias-gelu", action="store_true", help="bias-GELU backward instead of LN")
    args = ap.parse_args()
    C = _ext.load()
    tag = {k: os.environ.get(k, "default") for k in ("DCA_LN_BWD_RG", "DCA_LN_BWD_ROWS", "DCA_LN_BWD_BLOCKS",
                                                     "DCA_BGB_BLOCKS")}
    if args.bias_gelu:
        # MLP bias-GELU backward at d_ff = 4 x d_model: dy, x read, dx written, bias grad reduced
        for N in (3072, 4096, 6400):
            rows = args.rows
            dy = torch.randn(rows, N, device="cuda").bfloat16()
            x = torch.randn(rows, N, device="cuda").bfloat16()
            bias = torch.randn(N, device="cuda").bfloat16()
            acc = torch.zeros(N, device="cuda").bfloat16()
            ms = timeit(lambda: C.bias_gelu_bwd(dy, x, bias, True, acc))
            print(json.dumps({"op": "bias_gelu_bwd", "N": N, "rows": rows, **tag, "us": round(ms * 1e3, 2),
                              "GBps": round(3 * rows * N * 2 / ms / 1e6, 1)}), flush=True)
        return
    for D in (int(d) for d in args.widths.split(",")):
        rows = args.rows
        x = torch.randn(rows, D, device="cuda").bfloat16()
        dy = torch.randn(rows, D, device="cuda").bfloat16()
        ds = torch.randn(rows, D, device="cuda").bfloat16()
        w = torch.rand(D, device="cuda") + 0.5
        b = torch.randn(D, device="cuda")
        _, _, mean, rstd = C.ln_fwd(x, None, w, b, 1e-5, False)
        gacc = torch.zeros(D, device="cuda")
        bacc = torch.zeros(D, device="cuda")
        cacc = torch.zeros(D, device="cuda").bfloat16()
        for colsum in (False, True):
            fn = lambda: C.ln_bwd(dy, x, w, mean, rstd, ds, True, gacc, bacc, cacc if colsum else None)  # noqa: E731
            ms = timeit(fn)
            print(json.dumps({"op": "ln_bwd", "D": D, "rows": rows, "colsum": colsum, **tag,
                              "us": round(ms * 1e3, 2), "GBps": round(4 * rows * D * 2 / ms / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
