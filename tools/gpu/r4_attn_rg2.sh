#!/bin/bash
# attention forward with two 32-row query groups per wave (DCA_ATTN_FWD_RG=2, D = 64): numerics
# with the variant forced, then throughput A/B against the default kernel on one box
set -o pipefail
O=gpurun_out/r4rg2
mkdir -p $O
DCA_ATTN_FWD_RG=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash or hf" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SH="16,1024,16,64;32,1024,16,64;8,2048,16,64"
for r in 1 2; do
  echo "## default r$r" >> $O/bench.log
  timeout -k 10 200 python tools/bench_attn.py --only fwd --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
  timeout -k 10 200 python tools/bench_attn.py --only fwd --noncausal --shapes "16,1024,16,64" >> $O/bench.log 2>&1 || exit 1
  echo "## rg2 r$r" >> $O/bench.log
  DCA_ATTN_FWD_RG=2 timeout -k 10 200 python tools/bench_attn.py --only fwd --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
  DCA_ATTN_FWD_RG=2 timeout -k 10 200 python tools/bench_attn.py --only fwd --noncausal --shapes "16,1024,16,64" >> $O/bench.log 2>&1 || exit 1
done
grep -E '^##|"pass"' $O/bench.log | cut -c1-150
