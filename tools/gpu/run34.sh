#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r34_prof -o gpt -- python tools/bench_gpt2.py --micro 16 --steps 5 --warmup 3 > gpurun_out/r34_prof.log 2>&1
