# round 5: GPT-2 step vs the split-K factor of the weight gradients (DCA_WGRAD_SPLITS)
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
for i in 1 2; do
  for s in 2 4 8; do
    DCA_WGRAD_SPLITS=$s timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_s${s}_$i.log 2>&1 || exit 1
  done
done
