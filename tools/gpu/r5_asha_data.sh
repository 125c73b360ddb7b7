# round 5: ASHA full search (one GPU) with batched fp16 CIFAR fetching (examples/cifar10_asha)
set -o pipefail
OUT=gpurun_out/r5a2
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 500 python tools/bench_asha.py --gpus 1 --trace > $OUT/asha.json 2> $OUT/asha.err || exit 1
