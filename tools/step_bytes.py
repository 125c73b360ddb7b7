"""Whole-step HBM-bytes roofline of the ResNet-50 bench from rocprofv3 PMC passes.

Input: the ``run_counter_collection.csv`` of a ``--pmc FETCH_SIZE`` pass and of a ``--pmc
WRITE_SIZE`` pass over ``bench.py`` (tools/gpu/r5_step_bytes.sh; one counter group per pass since
FETCH_SIZE alone takes 3 of the 4 TCC counters). Both are in KB per dispatch (L2 <-> fabric). The
last complete training step is the dispatches after the second-to-last group of optimizer
(``sgd_kernel``) launches; bytes are summed per kernel category (tools/analyze_trace.py) and the
step's byte floor is reported against the measured 6.16 TB/s copy / 6.91 TB/s read ceilings
(profiles/round4_hbm_streaming_ceilings.txt).

Usage: python tools/step_bytes.py FETCH.csv WRITE.csv [sgd_launches_per_step=2] [step_ms]
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from analyze_trace import category  # noqa: E402


def load(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(rows))
        name = r["Kernel_Name"]
        v = float(r["Counter_Value"])
        if did in rows:
            rows[did] = (name, rows[did][1] + v)
        else:
            rows[did] = (name, v)
    return [rows[k] for k in sorted(rows)]


def last_step(rows, per_step):
    marks = [i for i, (n, _) in enumerate(rows) if "sgd_kernel" in n]
    if len(marks) < 2 * per_step:
        return rows
    return rows[marks[-2 * per_step + per_step - 1] + 1: marks[-1] + 1]


def main():
    fe, wr = load(sys.argv[1]), load(sys.argv[2])
    per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    step_ms = float(sys.argv[4]) if len(sys.argv) > 4 else None
    fs, ws = last_step(fe, per_step), last_step(wr, per_step)
    cat_f, cat_w, top = defaultdict(float), defaultdict(float), defaultdict(float)
    for n, v in fs:
        cat_f[category(n)] += v * 1024
        top[n[:90]] += v * 1024
    for n, v in ws:
        cat_w[category(n)] += v * 1024
        top[n[:90]] += v * 1024
    tf, tw = sum(cat_f.values()), sum(cat_w.values())
    print(f"kernels in the last step: fetch pass {len(fs)}, write pass {len(ws)}")
    print(f"step bytes: read {tf / 1e9:.2f} GB, write {tw / 1e9:.2f} GB, total {(tf + tw) / 1e9:.2f} GB")
    print(f"byte floor at 6.16 TB/s (copy ceiling): {(tf + tw) / 6.16e9:.2f} ms;"
          f" at 6.91 TB/s (read ceiling): {(tf + tw) / 6.91e9:.2f} ms"
          + (f"; measured step {step_ms:.2f} ms" if step_ms else ""))
    print("\nby category (GB read, GB written, ms at 6.16 TB/s):")
    for c in sorted(set(cat_f) | set(cat_w), key=lambda c: -(cat_f[c] + cat_w[c])):
        print(f"  {c:40s} {cat_f[c] / 1e9:8.2f} {cat_w[c] / 1e9:8.2f} {(cat_f[c] + cat_w[c]) / 6.16e9:8.2f}")
    print("\ntop kernels by bytes (GB):")
    for n, v in sorted(top.items(), key=lambda kv: -kv[1])[:30]:
        print(f"  {v / 1e9:8.2f}  {n}")


if __name__ == "__main__":
    main()
