# wgrad side-stream diagnostic (flat grads) + standalone BN kernels at bs 1024 under rocprofv3 stats
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/s2b
mkdir -p $O
timeout -k 10 120 python3 tools/dbg/wgrad_noise.py > $O/wgrad_noise.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bn -o run --output-format csv -- python3 $ROOT/tools/bench_bn.py --batch 1024 > $O/bn.txt 2>&1 || exit $?
cd $ROOT && s=$(find $O/bn -name 'run_kernel_stats.csv' | head -1) && cp $s $O/bn_stats.csv && f=$(find $O/bn -name 'run_kernel_trace.csv' | head -1) && python3 - "$f" > $O/bn_per_launch.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "bn_" not in n:
        continue
    key = (n.split("(")[0][-60:], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k[0]:60s} grid=({k[1]},{k[2]}) n={len(v)} med_us={v[len(v)//2]:.1f}")
PY
rm -f $f
