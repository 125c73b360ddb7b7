#!/bin/bash
# LN affine hoist + fast GELU + bias-GELU-bwd unroll; attention fwd LDS double buffer (1 barrier/tile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_transformer_ops_gpu.py > gpurun_out/r35_pytest.txt 2>&1 &&
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/r35_attn.txt 2>&1 &&
timeout -k 10 120 python tools/bench_ops.py --batch 16 > gpurun_out/r35_ops.txt 2>&1 &&
timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/r35_gpt2.txt 2>&1
