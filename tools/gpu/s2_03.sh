#!/bin/bash
# BN tpr<=32 geometry + 1x1 conv library comparison per direction.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_03_pytest.txt 2>&1 &&
timeout -k 10 200 python tools/bench_bn.py > gpurun_out/s2_03_bn.txt 2>&1 &&
timeout -k 10 300 python tools/bench_conv_ops.py > gpurun_out/s2_03_convops.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_03_bench.txt 2>&1
