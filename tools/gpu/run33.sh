#!/bin/bash
# GPT-2-medium ZeRO-2 DeepSpeed bench (micro 16) after the attention/bf16-pack speedups + kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/r33_gpt2.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r33_prof -o gpt -- python tools/bench_gpt2.py --micro 16 --steps 5 --warmup 3 > gpurun_out/r33_prof.log 2>&1
