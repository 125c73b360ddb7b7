# round 6: ASHA trials/hr on the final tree (the example's full search, one GPU, 16 concurrent trials)
set -o pipefail
OUT=gpurun_out/r6t2
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 600 python tools/bench_asha.py --gpus 1 --trace > $OUT/asha.log 2>&1 || exit 1
