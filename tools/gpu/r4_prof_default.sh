#!/bin/bash
# rocprofv3 step breakdown of the ResNet-50 bench in its default configuration (per stream)
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r4prof/default -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/r4prof/bench_default.log 2>&1 || exit 1
cd $ROOT && f=$(find gpurun_out/r4prof/default -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel > gpurun_out/r4prof/breakdown_default.txt && rm -f $f || exit 1
grep -A 32 "weight-gradient kernels" gpurun_out/r4prof/breakdown_default.txt
head -75 gpurun_out/r4prof/breakdown_default.txt
