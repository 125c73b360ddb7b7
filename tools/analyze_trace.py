"""Summarise a rocprofv3 kernel trace over the last N training steps.

Steps are delimited by the fused SGD kernel (one launch per param group per step). Prints the
per-step GPU busy time and the top kernels by time, grouped into categories."""
import csv
import re
import sys
from collections import defaultdict


def category(name: str) -> str:
    n = name
    if "dca" in n and "conv_fwd_kernel" in n:
        return "dca conv igemm (fwd + stride-1 dgrad)"
    if "dca" in n and ("conv_wgrad_kernel" in n or "wgrad_reduce" in n):
        return "dca conv wgrad"
    if "dca" in n and "flip_transpose" in n:
        return "dca conv weight flip"
    if "bn_" in n and "dca" in n:
        return "dca BatchNorm(+add+ReLU)"
    if "dca" in n and ("sgd_kernel" in n or "adam_kernel" in n or "lamb_" in n or "sumsq" in n
                       or "norm_finalize" in n):
        return "dca optimizer"
    if "igemm_fwd" in n or "conv_fwd" in n or "ConvFwd" in n or ("fwd" in n and "conv" in n.lower()):
        return "conv fwd (MIOpen)"
    if "igemm_bwd" in n or "bwd_data" in n or ("conv" in n.lower() and "bwd" in n and "weight" not in n):
        return "conv bwd-data (MIOpen)"
    if "wrw" in n or "bwd_weight" in n:
        return "conv bwd-weight (MIOpen)"
    if "dca" in n and "attn" in n:
        return "dca flash attention"
    if "gemm" in n.lower() or "Cijk" in n:
        return "gemm (fc)"
    if "fillBuffer" in n or "copyBuffer" in n:
        return "memset/copy"
    if "elementwise" in n or "Functor" in n:
        return "torch elementwise"
    if "reduce" in n.lower():
        return "torch reduce"
    return "other"


def main(path: str, steps: int = 3, step_marker: str = "sgd_kernel", per_step: int = 2,
         neighbors: str = "", by_grid: str = "") -> None:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if step_marker in r["Kernel_Name"]]
    # the fused optimizer launches once per (dtype buffer, param group): `per_step` per step
    marks = marks[per_step - 1::per_step]
    if len(marks) < steps + 1:
        print("not enough steps in trace")
        return
    lo, hi = marks[-steps - 1] + 1, marks[-1] + 1
    seg = rows[lo:hi]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    by_cat = defaultdict(float)
    by_name = defaultdict(lambda: [0.0, 0])
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        by_cat[category(r["Kernel_Name"])] += d
        k = by_name[r["Kernel_Name"][:110]]
        k[0] += d
        k[1] += 1
    print(f"steps={steps} wall/step={(t1 - t0) / 1e6 / steps:.3f} ms  gpu-busy/step={busy / 1e6 / steps:.3f} ms "
          f"kernels/step={len(seg) / steps:.0f}")
    print("\nby category (ms/step):")
    for c, v in sorted(by_cat.items(), key=lambda x: -x[1]):
        print(f"  {c:32s} {v / steps:8.3f}  {100 * v / (busy / 1e6):5.1f}%")
    skey = "Stream_Id" if seg and "Stream_Id" in seg[0] else ("Queue_Id" if seg and "Queue_Id" in seg[0] else None)
    if skey:
        # per stream / queue: the training step's critical path is the main stream's busy time
        by_stream = defaultdict(lambda: defaultdict(float))
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            by_stream[r[skey]][category(r["Kernel_Name"])] += d
        print(f"\nby {skey} (ms/step busy; categories):")
        for sid, cats in sorted(by_stream.items(), key=lambda x: -sum(x[1].values())):
            tot = sum(cats.values()) / steps
            parts = ", ".join(f"{c} {v / steps:.1f}" for c, v in sorted(cats.items(), key=lambda x: -x[1])[:6])
            print(f"  {skey}={sid}: {tot:8.3f}  [{parts}]")
        # which weight-gradient kernels run on which stream, and what precedes them there
        wg = defaultdict(lambda: [0.0, 0])
        prev_on = {}
        for r in seg:
            sid = r[skey]
            if category(r["Kernel_Name"]).startswith("conv bwd-weight"):
                key = (sid, r["Kernel_Name"][:70], prev_on.get(sid, "-")[:50])
                wg[key][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                wg[key][1] += 1
            prev_on[sid] = r["Kernel_Name"]
        print(f"\nweight-gradient kernels by {skey} (ms/step, calls/step, preceded on that stream by):")
        for (sid, n, pv), (v, c) in sorted(wg.items(), key=lambda x: (x[0][0], -x[1][0]))[:30]:
            print(f"  {skey}={sid} {v / steps:7.3f} {c / steps:4.1f}  {n} | after: {pv}")
    print("\ntop kernels (ms/step, calls/step):")
    for n, (v, c) in sorted(by_name.items(), key=lambda x: -x[1][0])[:40]:
        print(f"  {v / steps:8.3f} {c / steps:5.0f}  {n}")
    if by_grid:
        # per-launch-shape times of the kernels matching `by_grid` (grid size identifies the layer)
        shapes = defaultdict(lambda: [0.0, 0])
        for r in seg:
            if by_grid in r["Kernel_Name"]:
                short = re.sub(r"\(.*", "", r["Kernel_Name"]).split("::")[-1][:40]
                key = (short, r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"))
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                shapes[key][0] += d
                shapes[key][1] += 1
        print(f"\nlaunch shapes of '{by_grid}' (us/launch, launches/step, us/step):")
        for (nm, gx, gy), (v, c) in sorted(shapes.items(), key=lambda x: -x[1][0]):
            print(f"  {v / c:8.1f} {c / steps:5.1f} {v / steps:8.1f}  {nm} grid=({gx},{gy})")
    if neighbors:
        # which kernels surround the launches matching `neighbors` (who issues them)
        ctx = defaultdict(int)
        for i, r in enumerate(seg):
            if neighbors in r["Kernel_Name"]:
                prev = seg[i - 1]["Kernel_Name"][:60] if i else "-"
                nxt = seg[i + 1]["Kernel_Name"][:60] if i + 1 < len(seg) else "-"
                ctx[(prev, nxt)] += 1
        print(f"\nneighbours of '{neighbors}' (count/step: previous | next):")
        for (p, n), c in sorted(ctx.items(), key=lambda x: -x[1])[:12]:
            print(f"  {c / steps:5.1f}  {p} | {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3,
         per_step=int(sys.argv[3]) if len(sys.argv) > 3 else 2,
         step_marker=sys.argv[4] if len(sys.argv) > 4 else "sgd_kernel",
         neighbors=sys.argv[5] if len(sys.argv) > 5 else "",
         by_grid=sys.argv[6] if len(sys.argv) > 6 else "")
