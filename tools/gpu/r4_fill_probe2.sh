#!/bin/bash
# who launches the small fp32 fills in the ResNet step (enclosing autograd node + shape)
set -o pipefail
mkdir -p gpurun_out/r4fill2
timeout -k 10 300 python tools/probe_op_stacks.py --op aten::fill_ > gpurun_out/r4fill2/fills.log 2>&1 || { tail -20 gpurun_out/r4fill2/fills.log; exit 1; }
tail -32 gpurun_out/r4fill2/fills.log
