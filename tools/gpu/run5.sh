set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/r5_bench_ops.txt 2>&1; echo "bench_ops rc=$?"
cat gpurun_out/r5_bench_ops.txt | tail -20
