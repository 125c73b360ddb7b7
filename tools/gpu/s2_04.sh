#!/bin/bash
# 1x1 conv library chooser: numerics + same-box A/B (autotune on/off, BN row cap 32/256).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s2_04_pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_04_bench_a.txt 2>&1 &&
DCA_CONV_AUTOTUNE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_04_bench_noauto.txt 2>&1 &&
DCA_BN_MAXTPR=256 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_04_bench_tpr256.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/s2_04_bench_b.txt 2>&1
