#!/bin/bash
# D=64 pipelined forward with its MFMA bursts at raised wave priority (DCA_ATTN_FWD_PRIO=1) vs
# default: numerics with the variant, then throughput alternating on one box
set -o pipefail
O=gpurun_out/r4prio
mkdir -p $O
DCA_ATTN_FWD_PRIO=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SH="16,1024,16,64;32,1024,16,64;8,2048,16,64"
for r in 1 2 3; do
  echo "## default r$r" >> $O/bench.log
  timeout -k 10 200 python tools/bench_attn.py --only fwd --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
  echo "## prio r$r" >> $O/bench.log
  DCA_ATTN_FWD_PRIO=1 timeout -k 10 200 python tools/bench_attn.py --only fwd --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
done
grep -E '^##|"pass"' $O/bench.log | cut -c1-140
