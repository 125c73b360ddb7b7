#!/bin/bash
# round-4 numbers for the SD-2-shaped UNet step, and a GPT-2-medium ZeRO-2 step breakdown
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4sdgpt
mkdir -p $O
timeout -k 10 400 python3 tools/bench_diffusion.py --steps 10 --warmup 3 > $O/sd.txt 2>&1 || { tail -20 $O/sd.txt; exit 1; }
grep '"metric"' $O/sd.txt | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 6 --warmup 3 > $O/gpt.log 2>&1 || exit 1
cd $ROOT && f=$(find $O/g -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 8 adam_kernel > $O/gpt_breakdown.txt && rm -f $f || exit 1
head -45 $O/gpt_breakdown.txt
