"""Eager vs HIP-graph replay of single ops (follow-up of tools/probe_graph_miopen.py): which
library call computes something different when it is captured. Prints the relative difference
per op and BLAS backend. Usage: python tools/probe_graph_ops.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def compare(name, fn):
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            ref = fn().float().clone()
    torch.cuda.current_stream().wait_stream(s)
    e2 = fn().float().clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-30)).item()  # noqa: E731
    print(f"{name:60s} eager-eager {rel(e2, ref):.2e}  eager-replay {rel(out.float(), ref):.2e}", flush=True)


def main():
    torch.manual_seed(0)
    d = torch.device("cuda")
    bf = torch.bfloat16
    cl = torch.channels_last
    cases = []
    for (n, c, h, w, k, st) in ((8, 512, 4, 4, 1024, 2), (8, 1024, 2, 2, 2048, 2), (8, 256, 8, 8, 512, 2),
                                (256, 1024, 14, 14, 2048, 2), (8, 64, 8, 8, 64, 1)):
        x = torch.randn(n, c, h, w, device=d).to(bf).contiguous(memory_format=cl)
        wt = (torch.randn(k, c, 1, 1, device=d) * 0.05).to(bf).contiguous(memory_format=cl)
        cases.append((f"conv1x1 fwd {n}x{c}x{h}x{w}->{k} s{st}", lambda x=x, wt=wt, st=st: F.conv2d(x, wt, stride=st)))
    for (m, kk, nn) in ((32, 512, 1024), (8, 1024, 2048), (128, 256, 512), (512, 64, 256), (8, 2048, 10)):
        a = torch.randn(m, kk, device=d).to(bf)
        b = torch.randn(nn, kk, device=d).to(bf)
        cases.append((f"mm {m}x{kk} @ {kk}x{nn}", lambda a=a, b=b: torch.mm(a, b.t())))
        dy = torch.randn(m, nn, device=d).to(bf)
        cases.append((f"mm^T (wgrad-like) {kk}x{m} @ {m}x{nn}", lambda a=a, dy=dy: torch.mm(a.t(), dy)))
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            print("blas", lib, "unavailable:", e)
            continue
        print("## preferred_blas_library =", lib, flush=True)
        for name, fn in cases:
            compare(name, fn)


if __name__ == "__main__":
    main()
