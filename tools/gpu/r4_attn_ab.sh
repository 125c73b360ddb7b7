#!/bin/bash
# attention: numerics + throughput of the current build
set -o pipefail
mkdir -p gpurun_out
python -c "from determined_clone_amd.ops import _ext; print(_ext.load().__file__)" &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_transformer_ops_gpu.py -k "flash" > gpurun_out/attn_tests.log 2>&1 &&
tail -2 gpurun_out/attn_tests.log &&
timeout -k 10 200 python tools/bench_attn.py --shapes "16,1024,16,64;32,1024,16,64;8,2048,16,64;4,4096,8,128" > gpurun_out/attn_bench.log 2>&1 &&
timeout -k 10 200 python tools/bench_attn.py --noncausal --shapes "16,1024,16,64;4,4096,8,128" >> gpurun_out/attn_bench.log 2>&1 &&
grep '"pass"' gpurun_out/attn_bench.log
