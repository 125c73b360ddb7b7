"""Micro-benchmarks of the transformer kernels vs the PyTorch-ROCm equivalents (GPT-2-medium
shapes). Prints one line per op: ours ms, torch ms, and achieved TFLOP/s or GB/s."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from determined_clone_amd.ops import transformer as T


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
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--seq", type=int, default=1024)
    p.add_argument("--heads", type=int, default=16)
    p.add_argument("--head-dim", type=int, default=64)
    a = p.parse_args()
    B, S, H, D = a.batch, a.seq, a.heads, a.head_dim
    res = []
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    flops_f = 4 * B * H * S * S * D / 2  # causal
    ours_f = timeit(lambda: T.flash_attention(q, k, v, causal=True))
    qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_(True) for t in (q, k, v))
    sdpa = lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)  # noqa: E731
    ref_f = timeit(sdpa)
    res.append(dict(op="attn_fwd", ours_ms=ours_f, torch_ms=ref_f, ours_tflops=flops_f / ours_f / 1e9,
                    torch_tflops=flops_f / ref_f / 1e9))
    o = T.flash_attention(q, k, v, causal=True)
    ours_b = timeit(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True))
    o2 = sdpa()
    gt = g.transpose(1, 2).contiguous()
    ref_b = timeit(lambda: torch.autograd.grad(o2, (qt, kt, vt), gt, retain_graph=True))
    res.append(dict(op="attn_bwd", ours_ms=ours_b, torch_ms=ref_b, ours_tflops=2.5 * flops_f / ours_b / 1e9,
                    torch_tflops=2.5 * flops_f / ref_b / 1e9))
    E = H * D
    x = torch.randn(B * S, E, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w, b = torch.ones(E, device="cuda"), torch.zeros(E, device="cuda")
    ours = timeit(lambda: T.layer_norm(x, w, b, 1e-5, residual=r))
    ref = timeit(lambda: F.layer_norm(x + r, (E,), w.bfloat16(), b.bfloat16()))
    gb = 4 * x.numel() * 2 / 1e9
    res.append(dict(op="add_layernorm_fwd", ours_ms=ours, torch_ms=ref, ours_gbs=gb / ours * 1e3))
    h = torch.randn(B * S, 4 * E, device="cuda", dtype=torch.bfloat16)
    bias = torch.zeros(4 * E, device="cuda")
    ours = timeit(lambda: T.bias_gelu(h, bias))
    ref = timeit(lambda: F.gelu(h + bias.bfloat16(), approximate="tanh"))
    res.append(dict(op="bias_gelu_fwd", ours_ms=ours, torch_ms=ref, ours_gbs=2 * h.numel() * 2 / 1e9 / ours * 1e3))
    for r_ in res:
        print(json.dumps({k_: (round(v_, 4) if isinstance(v_, float) else v_) for k_, v_ in r_.items()}))


if __name__ == "__main__":
    main()
