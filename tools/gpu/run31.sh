#!/bin/bash
# attention kernel baseline + PMC counters of the forward kernel
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/r31_attn.txt 2>&1 &&
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/r31_counters.txt 2>&1 ;
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU -d gpurun_out/r31_pmc -o pmc --output-format csv -- python tools/bench_attn.py --iters 3 --only fwd > gpurun_out/r31_pmc.log 2>&1
