#!/bin/bash
# projection-shortcut strided accumulate on the HIP kernel (default) vs ATen's strided add_
# (DCA_STRIDED_ACC=0): conv GPU tests, then the ResNet-50 step alternating on one box
set -o pipefail
O=gpurun_out/r4sacc
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_transformer_ops_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    DCA_STRIDED_ACC=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/bench$v.log 2>&1 || exit 1
    echo "## bench STRIDED_ACC=$v round $r: $(tail -1 $O/bench$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
