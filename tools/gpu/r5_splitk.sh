# round 5: GPT-2 step with / without the split-K weight gradients (DCA_WGRAD_SPLITK)
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
for i in 1 2; do
  DCA_WGRAD_SPLITK=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_nosplit_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_split_$i.log 2>&1 || exit 1
done
