#!/bin/bash
# BN row-tile kernels: numerics, per-shape bandwidth, bench step + kernel trace.
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_02_pytest.txt 2>&1 &&
timeout -k 10 200 python tools/bench_bn.py > gpurun_out/s2_02_bn.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_02_bench.txt 2>&1 &&
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/s2prof2 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 5 > $ROOT/gpurun_out/s2_02_prof_stdout.txt 2>&1
