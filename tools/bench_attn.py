"""Flash-attention kernel throughput (ours) at GPT shapes: one JSON line per (shape, pass).
Usage: python tools/bench_attn.py [--iters N] [--only fwd|bwd]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import transformer as T  # noqa: E402


def timeit(fn, iters, warmup=5):
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
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=30)
    p.add_argument("--only", default="")
    p.add_argument("--gpt2", action="store_true", help="only the GPT-2-medium shape (16x1024x16x64)")
    p.add_argument("--shapes", default="", help="B,S,H,D[;B,S,H,D...] instead of the defaults")
    p.add_argument("--noncausal", action="store_true")
    p.add_argument("--kv-heads", type=int, default=0, help="grouped-query K/V heads (0: = H)")
    a = p.parse_args()
    shapes = ((16, 1024, 16, 64), (8, 2048, 16, 64), (4, 4096, 8, 128))
    if a.shapes:
        shapes = tuple(tuple(int(v) for v in t.split(",")) for t in a.shapes.split(";"))
    causal = not a.noncausal
    # clocks up before the first measured shape (the first shape otherwise reads low)
    w = [torch.randn(16, 1024, 16, 64, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3)]
    wo = T.flash_attention(*w, causal=causal)
    timeit(lambda: torch.autograd.grad(wo, w, wo, retain_graph=True), 100)
    for B, S, H, D in shapes[:1] if a.gpt2 else shapes:
        hk = a.kv_heads or H
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k, v = (torch.randn(B, S, hk, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
                for _ in range(2))
        g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        flops = 4 * B * H * S * S * D / (2 if causal else 1)
        if a.only in ("", "fwd"):
            ms = timeit(lambda: T.flash_attention(q, k, v, causal=causal), a.iters)
            print(json.dumps({"B": B, "S": S, "H": H, "Hkv": hk, "D": D, "causal": causal, "pass": "fwd", "ms": round(ms, 4),
                              "tflops": round(flops / ms / 1e9, 1)}), flush=True)
        if a.only in ("", "bwd"):
            o = T.flash_attention(q, k, v, causal=causal)
            ms = timeit(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True), a.iters)
            print(json.dumps({"B": B, "S": S, "H": H, "Hkv": hk, "D": D, "causal": causal, "pass": "bwd", "ms": round(ms, 4),
                              "tflops": round(2.5 * flops / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
