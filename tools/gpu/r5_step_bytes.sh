# whole-step HBM bytes of the default ResNet-50 bench (bs 1024) from PMC FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r5_bytes
mkdir -p $OUT
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 > $OUT/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 1 > $OUT/write.log 2>&1 && \
cd $ROOT && python3 tools/step_bytes.py $(find $OUT/fetch -name 'run_counter_collection.csv' | head -1) $(find $OUT/write -name 'run_counter_collection.csv' | head -1) 2 78.1 > $OUT/summary.txt 2>&1; \
find $OUT -name '*.csv' -size +20M -delete
# GPT-2 kernel trace: are there device copies inside the steady-state step?
mkdir -p $ROOT/gpurun_out/r5_gpt2 && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r5_gpt2/prof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 6 --warmup 3 > $ROOT/gpurun_out/r5_gpt2/bench.log 2>&1 && \
cd $ROOT && f=$(find gpurun_out/r5_gpt2/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 9 adam_kernel copyBuffer > gpurun_out/r5_gpt2/breakdown.txt && \
s=$(find gpurun_out/r5_gpt2/prof -name 'run_kernel_stats.csv' | head -1) && head -45 $s > gpurun_out/r5_gpt2/kernel_stats_head.csv && rm -f $f
