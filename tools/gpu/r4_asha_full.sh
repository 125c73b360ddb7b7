#!/bin/bash
# ASHA trials/hr at the example's full search config on one MI355X (16 concurrent trials on 16 slots)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u tools/bench_asha.py --gpus 1 --trace --timeout 1000 > gpurun_out/asha_full.json 2> gpurun_out/asha_full.log
rc=$?
tail -3 gpurun_out/asha_full.log; cat gpurun_out/asha_full.json
exit $rc
