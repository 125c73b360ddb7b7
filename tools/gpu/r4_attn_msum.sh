#!/bin/bash
# forward row sums on the matrix core (DCA_ATTN_FWD_MSUM): numerics + same-box A/B
set -o pipefail
mkdir -p gpurun_out
DCA_ATTN_FWD_MSUM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_transformer_ops_gpu.py -k "flash" > gpurun_out/msum_tests.log 2>&1 && tail -1 gpurun_out/msum_tests.log &&
for r in 1 2; do for v in 0 1; do
  echo "## MSUM=$v round $r" >> gpurun_out/msum_ab.log
  DCA_ATTN_FWD_MSUM=$v timeout -k 10 200 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" >> gpurun_out/msum_ab.log 2>&1 || exit 1
  DCA_ATTN_FWD_MSUM=$v timeout -k 10 200 python tools/bench_attn.py --only fwd --noncausal --shapes "16,1024,16,64;4,4096,8,128" >> gpurun_out/msum_ab.log 2>&1 || exit 1
done; done
grep -E "^##|\"pass\"" gpurun_out/msum_ab.log | cut -c1-140
