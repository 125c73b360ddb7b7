# rocprofv3 kernel trace of the ResNet-50 bench; which kernels surround MIOpen's SubTensorOpWithScalar1d
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/nb
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/nb/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/nb/prof_bench.log 2>&1 && \
cd $ROOT && f=$(find gpurun_out/nb/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel SubTensorOpWithScalar1d > gpurun_out/nb/neighbors.txt && \
python3 - "$f" > gpurun_out/nb/subtensor_sizes.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
c = collections.Counter()
for i, r in enumerate(rows):
    if "SubTensorOpWithScalar1d" in r["Kernel_Name"]:
        nxt = rows[i + 1]["Kernel_Name"][:90] if i + 1 < len(rows) else ""
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c[(r.get("Grid_Size_X", r.get("Grid_Size", "")), round(dur, -1), nxt)] += 1
for k, v in c.most_common(40):
    print(v, k)
PY
rm -f $f
