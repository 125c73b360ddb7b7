#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_pipeline_gpu.py tests/test_distributed_gpu.py tests/test_graph_gpu.py tests/test_ops_gpu.py \
  > gpurun_out/r29_pytest.txt 2>&1
