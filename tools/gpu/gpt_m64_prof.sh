# why GPT-2-medium ZeRO-2 collapses at micro 64 (755 ms/step vs 93 at 32): kernel stats
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/m64
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/m64/prof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --micro 64 --steps 3 --warmup 2 > $ROOT/gpurun_out/m64/bench.log 2>&1 && \
cd $ROOT && s=$(find gpurun_out/m64/prof -name 'run_kernel_stats.csv' | head -1) && head -25 $s | cut -c1-250 > gpurun_out/m64/stats_head.txt && \
f=$(find gpurun_out/m64/prof -name 'run_kernel_trace.csv' | head -1) && rm -f $f
