# round 5: measure + ship the conv chooser decisions, check a bench run times nothing, ASHA start-up marks
set -o pipefail
mkdir -p gpurun_out/r5c
( while sleep 30; do date +%T >> gpurun_out/r5c/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u tools/dump_conv_choices.py --out gpurun_out/r5c/conv_choices_gfx950.json > gpurun_out/r5c/dump.log 2>&1 && \
DCA_CONV_CHOICES=gpurun_out/r5c/conv_choices_gfx950.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5c/bench_shipped.log 2>&1 && \
timeout -k 10 400 python tools/bench_asha.py --gpus 1 --trace > gpurun_out/r5c/asha.log 2>&1
