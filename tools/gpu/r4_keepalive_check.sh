#!/bin/bash
# side-stream keepalive: GPU tests of the gradient paths + bench memory diagnostics
set -o pipefail
mkdir -p gpurun_out
python -c "from determined_clone_amd.ops import _ext; print(_ext.load().__file__)" &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_conv_gpu.py tests/test_graph_gpu.py > gpurun_out/keepalive_tests.log 2>&1 &&
tail -3 gpurun_out/keepalive_tests.log &&
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/keepalive_bench.json 2> gpurun_out/keepalive_bench.err &&
cat gpurun_out/keepalive_bench.json && grep step_ms gpurun_out/keepalive_bench.err
