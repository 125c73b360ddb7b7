#!/bin/bash
# per-kernel bandwidth of the BN kernels at every ResNet-50 shape (bs 1024)
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/bnk
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/bnk/t -o run -- python3 $ROOT/tools/bench_bn_kernels.py --run > $ROOT/gpurun_out/bnk/run.log 2>&1 || exit 1
cd $ROOT && f=$(find gpurun_out/bnk/t -name 'run_kernel_trace.csv' | head -1) && python3 tools/bench_bn_kernels.py --trace $f > gpurun_out/bnk/summary.txt && rm -f $f && cat gpurun_out/bnk/summary.txt
