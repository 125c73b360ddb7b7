# GPT-2-medium ZeRO-2 at the default micro 32: kernel stats
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/m32
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/m32/prof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --micro 32 --steps 4 --warmup 3 > $ROOT/gpurun_out/m32/bench.log 2>&1 && \
cd $ROOT && s=$(find gpurun_out/m32/prof -name 'run_kernel_stats.csv' | head -1) && head -25 $s | cut -c1-250 > gpurun_out/m32/stats_head.txt && \
f=$(find gpurun_out/m32/prof -name 'run_kernel_trace.csv' | head -1) && rm -f $f
