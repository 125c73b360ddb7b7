"""Per-dispatch view of one training step from a rocprofv3 kernel trace: every kernel of the last
step in launch order with its duration, grid and a short name (used to price the BN kernels and
the small glue kernels per ResNet-50 layer)."""
import csv
import re
import sys


def short(n: str) -> str:
    m = re.search(r"dca::\(anonymous namespace\)::(\w+)", n)
    if m:
        return m.group(1) + ("<bwd>" if ("true>" in n[:160] or "true," in n[:160]) else "")
    return n[:60]


def main(path: str, marker: str = "sgd_kernel") -> None:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = marks[-3] + 1, marks[-1] + 1  # last step (2 optimizer launches per step)
    tot = 0
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]))
        print(f"{d:9.1f} us  wg={grid:6d}  {short(r['Kernel_Name'])}")
    print(f"total {tot / 1e3:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
