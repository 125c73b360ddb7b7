#!/bin/bash
# BN statistics (reduce) passes: channel-group-fastest flat grid (default) vs the 2-D grid (DCA_BN_REDUCE_FLAT=0):
# numerics, per-kernel bandwidth at every ResNet-50 BN shape, and the ResNet-50 step, same box
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4bnrflat
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_conv_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  cd /tmp && DCA_BN_REDUCE_FLAT=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$v -o run -- python3 $ROOT/tools/bench_bn_kernels.py --run > $O/run$v.log 2>&1 || exit 1
  cd $ROOT && f=$(find $O/t$v -name 'run_kernel_trace.csv' | head -1) && python3 tools/bench_bn_kernels.py --trace $f > $O/summary$v.txt && rm -f $f || exit 1
  echo "## FLAT=$v"; grep -E '"C": (1024|2048|512)|per_step' $O/summary$v.txt
done
for r in 1 2; do
  for v in 1 0; do
    DCA_BN_REDUCE_FLAT=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/bench$v.log 2>&1 || exit 1
    echo "## bench FLAT=$v round $r: $(tail -1 $O/bench$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
