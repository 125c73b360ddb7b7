# round 5 first call: baseline bench on this session's box + GPT-2 D2D copy attribution
set -o pipefail
mkdir -p gpurun_out/r5a
( while sleep 30; do date +%T >> gpurun_out/r5a/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5a/bench.log 2>&1 && \
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > gpurun_out/r5a/gpt2.log 2>&1 && \
timeout -k 10 300 python tools/probe_gpt2_copies.py --steps 2 > gpurun_out/r5a/gpt2_copies.txt 2>&1
