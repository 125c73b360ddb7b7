"""Per-kernel HBM bandwidth of the fused BatchNorm(+ReLU) kernels at every ResNet-50 BN shape.

Run under ``rocprofv3 --kernel-trace --output-format csv`` (``--run``), then summarise the trace
(``--trace <csv>``): each shape's launches sit between two marker kernels (``torch.cuda._sleep``,
ATen's spin kernel), so every kernel of every shape gets its own time and, from the tensor sizes,
its achieved bandwidth. Bytes counted per kernel: reduce fwd reads x; apply fwd reads x, writes y
and the ReLU bitmask; reduce bwd reads x, dy and the bitmask; apply bwd reads x, dy, the bitmask
and writes dx (no residual in this benchmark).

Usage: rocprofv3 --kernel-trace --output-format csv -d D -o run -- python tools/bench_bn_kernels.py --run
       python tools/bench_bn_kernels.py --trace D/.../run_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

# (C, H, W, count in ResNet-50 per step)
SHAPES = [(64, 56, 56, 6), (256, 56, 56, 4), (128, 56, 56, 1), (128, 28, 28, 7), (512, 28, 28, 5),
          (256, 28, 28, 1), (256, 14, 14, 11), (1024, 14, 14, 7), (512, 14, 14, 1), (512, 7, 7, 5),
          (2048, 7, 7, 4)]


def run(batch: int, iters: int) -> None:
    import torch

    from determined_clone_amd.ops import batchnorm as bn

    dev = torch.device("cuda")
    for C, H, W, _ in SHAPES:
        x = torch.randn(batch, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        w = torch.ones(C, device=dev, requires_grad=True)
        b = torch.zeros(C, device=dev, requires_grad=True)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        g = torch.randn(batch, C, H, W, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        for _ in range(2):  # warm-up
            bn.batch_norm_act(x, w, b, rm, rv).backward(g)
        torch.cuda.synchronize()
        torch.cuda._sleep(1000)  # segment start marker
        for _ in range(iters):
            bn.batch_norm_act(x, w, b, rm, rv).backward(g)
        torch.cuda._sleep(1000)  # segment end marker
        torch.cuda.synchronize()
        del x, g
        torch.cuda.empty_cache()
    print("done", flush=True)


def kind(name: str) -> str:
    if "bn_reduce_kernel" in name:
        return "reduce_bwd" if ", true," in name else "reduce_fwd"
    if "bn_apply_fwd" in name:
        return "apply_fwd"
    if "bn_apply_bwd" in name:
        return "apply_bwd"
    if "finalize" in name:
        return "finalize_bwd" if "bwd" in name else "finalize_fwd"
    return ""


def summarise(path: str, batch: int) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "spin_kernel" in n or "sleep" in n.lower():
            if cur is None:
                cur = defaultdict(list)
            else:
                segs.append(cur)
                cur = None
            continue
        if cur is not None:
            k = kind(n)
            if k:
                cur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = defaultdict(float)
    out = []
    for (C, H, W, cnt), seg in zip(SHAPES, segs):
        n = batch * C * H * W
        t = 2 * n  # bytes of one bf16 tensor
        m = n // 8  # ReLU bitmask
        nbytes = {"reduce_fwd": t, "apply_fwd": 2 * t + m, "reduce_bwd": 2 * t + m, "apply_bwd": 3 * t + m}
        res = {"C": C, "HW": f"{H}x{W}", "MB": round(t / 1e6, 1)}
        for k, v in sorted(seg.items()):
            us = sorted(v)[len(v) // 2]
            res[k + "_us"] = round(us, 1)
            if k in nbytes:
                res[k + "_TBps"] = round(nbytes[k] / us / 1e6, 2)
            tot[k] += us * cnt
        out.append(res)
        print(json.dumps(res), flush=True)
    print(json.dumps({"per_step_ms_at_batch": batch, **{k: round(v / 1e3, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--trace")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    if a.run:
        run(a.batch, a.iters)
    if a.trace:
        summarise(a.trace, a.batch)
