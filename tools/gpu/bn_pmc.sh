# HBM bytes of the fused BatchNorm kernels from PMC counters (TCC FETCH_SIZE / WRITE_SIZE, one
# counter per pass: the TCC block holds 4 and FETCH_SIZE alone uses 3), ResNet-50 bench bs 256
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/bn_pmc
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $ROOT/gpurun_out/bn_pmc/fetch -o run --output-format csv -- python3 $ROOT/bench.py --batch 256 --steps 2 --warmup 1 > $ROOT/gpurun_out/bn_pmc/fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $ROOT/gpurun_out/bn_pmc/write -o run --output-format csv -- python3 $ROOT/bench.py --batch 256 --steps 2 --warmup 1 > $ROOT/gpurun_out/bn_pmc/write.log 2>&1 && \
cd $ROOT && python3 - > gpurun_out/bn_pmc/summary.txt <<'PY'
import csv, glob, collections, re
def load(kind):
    f = glob.glob(f"gpurun_out/bn_pmc/{kind}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "bn_" not in name:
            continue
        m = re.search(r"(bn_[a-z_]+_kernel<[^>(]*>?)", name)
        short = m.group(1) if m else name[:60]
        agg[(short, r.get("Grid_Size", ""))].append(float(r["Counter_Value"]))
    return agg
fe, wr = load("fetch"), load("write")
print("kernel, grid, launches, mean FETCH_SIZE MB, mean WRITE_SIZE MB")
for k in sorted(fe, key=lambda k: -sum(fe[k])):
    w = wr.get(k, [0.0])
    print(f"{k[0]}, {k[1]}, {len(fe[k])}, {sum(fe[k]) / len(fe[k]) / 1024:.1f}, {sum(w) / len(w) / 1024:.1f}")
PY
find gpurun_out/bn_pmc -name '*.csv' -size +20M -delete
