# round 5: ASHA full search on one GPU, trials with and without the HIP-graph-captured step
set -o pipefail
OUT=gpurun_out/r5t
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 500 python tools/bench_asha.py --gpus 1 --hip-graph 1 > $OUT/asha_graph.json 2> $OUT/asha_graph.err || exit 1
timeout -k 10 500 python tools/bench_asha.py --gpus 1 --hip-graph 0 > $OUT/asha_eager.json 2> $OUT/asha_eager.err || exit 1
