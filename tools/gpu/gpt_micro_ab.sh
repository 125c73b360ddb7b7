# GPT-2-medium ZeRO-2 DeepSpeedTrial: tokens/s at micro batch 16 / 32 / 64 per GPU (288 GB HBM)
set -o pipefail
mkdir -p gpurun_out/gpt_micro
for m in 16 32 64 16; do
  timeout -k 10 300 python tools/bench_gpt2.py --micro $m --steps 10 --warmup 4 > gpurun_out/gpt_micro/m$m.$RANDOM.txt 2>&1 || exit 1
done
