#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -m gpu tests/test_zero3.py tests/test_pipeline_gpu.py > gpurun_out/r30_pytest.txt 2>&1
