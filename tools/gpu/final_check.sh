# round-end style check: GPU tests, default bench (bs 1024/GPU), smoke, then a rocprofv3 kernel
# trace of the bench with the per-step breakdown (tools/analyze_trace.py)
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/final
( while sleep 30; do date +%T >> gpurun_out/final/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 && \
export TMPDIR=/tmp && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/final/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/final/prof_bench.log 2>&1 && \
cd $ROOT && f=$(find gpurun_out/final/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > gpurun_out/final/resnet_breakdown.txt && \
s=$(find gpurun_out/final/prof -name 'run_kernel_stats.csv' | head -1) && head -40 $s > gpurun_out/final/kernel_stats_head.csv && \
rm -f $f
