#!/bin/bash
# attention dK/dV kernel Q/dO prefetch through buffer descriptors: numerics + A/B vs ab/_C_old.so
# (same box, alternating); then who launches the small fp32 fills in the ResNet step
set -o pipefail
mkdir -p gpurun_out/r4attn3
O=gpurun_out/r4attn3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_transformer_ops_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SH="16,1024,16,64;8,2048,16,64;4,4096,8,128"
for r in 1 2; do
  echo "## old round $r" >> $O/bench.log
  DCA_OPS_SO=$PWD/ab/_C_old.so timeout -k 10 200 python tools/bench_attn.py --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
  echo "## new round $r" >> $O/bench.log
  timeout -k 10 200 python tools/bench_attn.py --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
done
grep -E '^##|"pass"' $O/bench.log
timeout -k 10 300 python tools/probe_op_stacks.py --op aten::fill_ > $O/fills.log 2>&1 || { tail -20 $O/fills.log; exit 1; }
tail -25 $O/fills.log
