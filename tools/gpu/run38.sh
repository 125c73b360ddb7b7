#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_transformer_ops_gpu.py tests/test_gpt2.py > gpurun_out/r38_pytest.txt 2>&1 &&
timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/r38_gpt2.txt 2>&1
