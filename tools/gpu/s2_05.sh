#!/bin/bash
# dual pointwise (strided shortcut dgrad), avgpool bwd kernel: numerics + same-box A/B + trace
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_05_pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_05_bench_a.txt 2>&1 &&
DCA_PW_DUAL=0 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_05_bench_nodual.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_05_bench_b.txt 2>&1 &&
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/s2prof5 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 5 > $ROOT/gpurun_out/s2_05_prof_stdout.txt 2>&1
