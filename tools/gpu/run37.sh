#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_transformer_ops_gpu.py > gpurun_out/r37_pytest.txt 2>&1 &&
timeout -k 10 120 python tools/bench_attn.py --only fwd > gpurun_out/r37_attn.txt 2>&1 &&
timeout -k 10 120 python tools/bench_wgrad.py > gpurun_out/r37_wgrad.txt 2>&1
