#!/bin/bash
# conv GPU tests, then a rocprof step breakdown with the FillFunctor<float> launches' grid sizes
# and neighbours (who issues them) -- after ctx.set_materialize_grads(False) in ops/conv.py
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4fill
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -m gpu > gpurun_out/r4fill/tests.log 2>&1 || { tail -30 gpurun_out/r4fill/tests.log; exit 1; }
tail -2 gpurun_out/r4fill/tests.log
timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/r4fill/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r4fill/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r4fill/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/r4fill/bench_prof.log 2>&1 || exit 1
cd $ROOT && f=$(find gpurun_out/r4fill/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "FillFunctor<float>" "FillFunctor<float>" > gpurun_out/r4fill/breakdown.txt && rm -f $f || exit 1
head -20 gpurun_out/r4fill/breakdown.txt
grep -A 14 "neighbours of" gpurun_out/r4fill/breakdown.txt
grep -A 14 "launch shapes of" gpurun_out/r4fill/breakdown.txt
