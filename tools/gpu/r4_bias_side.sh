#!/bin/bash
# linear bias gradients on the side stream (default) vs on the data-gradient stream
# (DCA_BIAS_GRAD_SIDE=0): GPU tests touching the linear / GPT paths, then the GPT-2-medium
# ZeRO-2 step alternating on one box
set -o pipefail
O=gpurun_out/r4bias
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread $(grep -l "linear\|gpt\|GPT" tests/test_*gpu*.py) > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    DCA_BIAS_GRAD_SIDE=$v timeout -k 10 240 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt$v.log 2>&1 || exit 1
    echo "## gpt2 BIAS_GRAD_SIDE=$v round $r: $(grep '"metric"' $O/gpt$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
