#!/bin/bash
# ResNet-50 step with the weight-gradient side stream restricted to half of the CUs
# (DCA_WGRAD_CU_MASK) vs unrestricted; alternating on one box
set -o pipefail
O=gpurun_out/r4cumask
mkdir -p $O
DCA_WGRAD_CU_MASK=even timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "side or keepalive or wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in none even lo 64; do
    if [ $v = none ]; then E="DCA_X=0"; else E="DCA_WGRAD_CU_MASK=$v"; fi
    env $E timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/b_$v.txt 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    echo "## CU_MASK=$v round $r: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d["value"], d["ms_per_step"])' $O/b_$v.txt)"
  done
done
