#!/bin/bash
# isolated forward vs stride-1 data-gradient timing of the implicit-GEMM 3x3 convolutions (bs 1024):
# in the full step the data gradients take ~2x the forward per call, while the side-stream weight
# gradients share the chip -- this separates kernel cost from contention
set -o pipefail
O=gpurun_out/r4igiso
mkdir -p $O
timeout -k 10 400 python3 tools/bench_igemm.py --batch 1024 > $O/bench_igemm.txt 2>&1 || { tail -20 $O/bench_igemm.txt; exit 1; }
grep -v "^\s*$" $O/bench_igemm.txt | tail -30 | cut -c1-250
