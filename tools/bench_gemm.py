"""The large-tile MFMA GEMM (csrc/gemm.hip) against hipBLASLt (torch F.linear) on the GPT-2-medium
projection shapes at micro batch 32 x seq 1024, plus the fused MLP backward (gemm_nt_dgelu) against
hipBLASLt + bias_gelu_bwd. One JSON line per shape: median of --iters (HIP events), same process,
interleaved rounds."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

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
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    C = _ext.load()
    T = args.tokens
    # (name, N, K): forward projections y = x W^T (W [N, K]) and data gradients dx = dy W (B = W^T)
    shapes = [("qkv", 3072, 1024), ("attn_out", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
              ("fc1_dgrad", 1024, 4096), ("qkv_dgrad", 1024, 3072)]
    for rnd in range(args.rounds):
        for name, N, K in shapes:
            a = torch.randn(T, K, device="cuda").bfloat16()
            b = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
            bias = torch.randn(N, device="cuda").bfloat16()
            flops = 2 * T * N * K
            ours = timeit(lambda: C.gemm_nt(a, b, bias), args.iters)
            lt = timeit(lambda: F.linear(a, b, bias), args.iters)
            err = ((C.gemm_nt(a, b, bias).float() - F.linear(a, b, bias).float()).norm()
                   / F.linear(a, b, bias).float().norm()).item()
            print(json.dumps({"round": rnd, "shape": name, "M": T, "N": N, "K": K, "ours_us": round(ours, 1),
                              "ours_tf": round(flops / ours / 1e6, 1), "hipblaslt_us": round(lt, 1),
                              "hipblaslt_tf": round(flops / lt / 1e6, 1), "rel_diff": round(err, 5)}), flush=True)
        for E, Fd in ((1024, 4096),):
            dy = torch.randn(T, E, device="cuda").bfloat16()
            w2 = (torch.randn(E, Fd, device="cuda") * E ** -0.5).bfloat16()
            w2t = w2.t().contiguous()
            z = torch.randn(T, Fd, device="cuda").bfloat16()
            bb = torch.randn(Fd, device="cuda") * 0.5
            fused = timeit(lambda: C.gemm_nt_dgelu(dy, w2t, z, bb), args.iters)
            dh = dy @ w2
            unf = timeit(lambda: dy @ w2, args.iters) + timeit(
                lambda: C.bias_gelu_bwd(dh, z, bb, True, None), args.iters)
            print(json.dumps({"round": rnd, "shape": "mlp_dgelu", "M": T, "N": Fd, "K": E, "fused_us": round(fused, 1),
                              "fused_tf": round(2 * T * E * Fd / fused / 1e6, 1), "unfused_us": round(unf, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
