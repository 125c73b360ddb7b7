#!/bin/bash
# GPT-2-medium ZeRO-2: the last N weight gradients of each backward pass on the data-gradient
# stream (DCA_WGRAD_MAIN_TAIL=N) instead of the side stream; alternating on one box
set -o pipefail
O=gpurun_out/r4tail
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_transformer_ops_gpu.py -k "direct_grad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 0 8 16 32; do
    DCA_WGRAD_MAIN_TAIL=$v timeout -k 10 240 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt$v.log 2>&1 || exit 1
    echo "## gpt2 MAIN_TAIL=$v round $r: $(grep '"metric"' $O/gpt$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
