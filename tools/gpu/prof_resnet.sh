# rocprofv3 kernel trace of the ResNet-50 bench + per-step breakdown (run via gpurun)
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/prof_bench.log 2>&1 && \
cd $ROOT && f=$(find gpurun_out/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > gpurun_out/resnet_breakdown.txt && head -1 $f > gpurun_out/trace_header.txt && \
rm -f $f
