#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/conv_det_prof -o conv_det -- python3 tools/probe_conv_det.py > gpurun_out/conv_det.txt 2>&1 &&
timeout -k 10 120 python3 tools/probe_conv_det.py --det >> gpurun_out/conv_det.txt 2>&1 &&
MIOPEN_LOG_LEVEL=6 timeout -k 10 120 python3 tools/probe_conv_det.py >> gpurun_out/conv_det_log.txt 2>&1
rc=$?
grep "deterministic=" gpurun_out/conv_det.txt
find gpurun_out/conv_det_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-4 {} | head -12
grep -E "algorithm|algo =|Solver|olver" gpurun_out/conv_det_log.txt | sort | uniq -c | head
exit $rc
