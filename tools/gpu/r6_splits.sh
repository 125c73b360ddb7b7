# round 6: GPT-2 linear weight-gradient split-K factor A/B at 32k tokens per step
set -o pipefail
OUT=gpurun_out/r6l2
mkdir -p $OUT
for i in 1 2; do
  for s in 4 8; do
    timeout -k 10 300 python tools/probe_wgrad_splits.py $s --steps 10 --warmup 3 > $OUT/split${s}_$i.log 2>&1 || exit 1
  done
done
