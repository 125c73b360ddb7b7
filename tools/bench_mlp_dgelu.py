"""GPT-2 MLP backward through the projection and the GELU: the fused ``linear_dgelu`` kernel
(implicit-GEMM MFMA kernel with the dGELU + bias-partials epilogue) against hipBLASLt's dH = dY W
followed by ``bias_gelu_bwd``. Prints one JSON line per shape (median of --iters, HIP events)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from determined_clone_amd.ops import _ext  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[iters // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    C = _ext.load()
    for E, F in ((1024, 4096), (768, 3072)):
        T = args.tokens
        dy = torch.randn(T, E, device="cuda").bfloat16()
        w = (torch.randn(E, F, device="cuda") * E ** -0.5).bfloat16()
        z = torch.randn(T, F, device="cuda").bfloat16()
        b = torch.randn(F, device="cuda") * 0.5
        flops = 2 * T * E * F
        t_fused = timeit(lambda: C.linear_dgelu(dy, w, z, b), args.iters)
        t_gemm = timeit(lambda: dy @ w, args.iters)
        dh = dy @ w
        t_gelu = timeit(lambda: C.bias_gelu_bwd(dh, z, b, True, None), args.iters)
        t_tr = timeit(lambda: w.t().contiguous(), args.iters)
        print(json.dumps({"T": T, "E": E, "F": F, "fused_us": round(t_fused, 1),
                          "fused_tf": round(flops / t_fused / 1e6, 1), "lt_gemm_us": round(t_gemm, 1),
                          "lt_tf": round(flops / t_gemm / 1e6, 1), "bias_gelu_bwd_us": round(t_gelu, 1),
                          "unfused_us": round(t_gemm + t_gelu, 1), "transpose_us": round(t_tr, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
