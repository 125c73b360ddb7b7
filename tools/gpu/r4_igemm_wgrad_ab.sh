#!/bin/bash
# ResNet-50: every eligible weight gradient on the implicit-GEMM kernel (DCA_IGEMM_WGRAD=1) vs the
# per-shape chooser (auto) vs MIOpen only (0); alternating on one box
set -o pipefail
O=gpurun_out/r4igw
mkdir -p $O
for r in 1 2; do
  for v in auto 1 0; do
    DCA_IGEMM_WGRAD=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/b_$v.txt 2> $O/b_$v.err || { tail -5 $O/b_$v.err; exit 1; }
    echo "## IGEMM_WGRAD=$v round $r: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d["value"], d["ms_per_step"])' $O/b_$v.txt)"
  done
done
