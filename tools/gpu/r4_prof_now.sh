#!/bin/bash
# rocprof step breakdown of the current default ResNet-50 bench (per stream, top kernels,
# neighbours of the strided elementwise kernels)
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4profnow
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $O/bench.log 2>&1 || exit 1
cd $ROOT && f=$(find $O/t -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "elementwise_kernel_manual_unroll" "Functor" > $O/breakdown.txt && rm -f $f || exit 1
head -75 $O/breakdown.txt
grep -A 14 "neighbours of" $O/breakdown.txt
grep -A 20 "launch shapes of" $O/breakdown.txt
