# round 5: bias-GELU backward row-slab sweep (micro), GPT-2 A/B row-group LN backward vs the old
# kernel at the shipped defaults, and a ResNet-50 sanity bench
set -o pipefail
OUT=gpurun_out/r5i
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
for b in 256 512 1024 2048; do
  DCA_BGB_BLOCKS=$b timeout -k 10 120 python tools/bench_ln_bwd.py --bias-gelu >> $OUT/bgb.jsonl 2>>$OUT/bgb.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_rg_$i.log 2>&1 || exit 1
  DCA_LN_BWD_RG=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_old_$i.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/rn.log 2>&1 || exit 1
