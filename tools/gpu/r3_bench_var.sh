set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
O=gpurun_out/r3
(rocm-smi --showclocks --showpower --showtemp --showperflevel --showuse > $O/smi_before.txt 2>&1 || true)
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit $?
  (rocm-smi --showclocks --showpower --showtemp > $O/smi_after_$i.txt 2>&1 || true)
done
grep -h metric $O/bench_*.log
