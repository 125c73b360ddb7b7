# round 5: row-group LayerNorm backward -- numerics, then a knob sweep of the micro-benchmark and a
# GPT-2 A/B (old one-row-per-wave kernel vs row-group kernel)
set -o pipefail
OUT=gpurun_out/r5g
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py \
  -k "layer_norm or ln_bwd or out_projection" > $OUT/pytest.log 2>&1 || exit 1
DCA_LN_BWD_RG=0 timeout -k 10 120 python tools/bench_ln_bwd.py > $OUT/sweep.jsonl 2>$OUT/sweep.err || exit 1
for r in 2 4; do for b in 256 512 1024 2048; do
  DCA_LN_BWD_ROWS=$r DCA_LN_BWD_BLOCKS=$b timeout -k 10 120 python tools/bench_ln_bwd.py >> $OUT/sweep.jsonl 2>>$OUT/sweep.err || exit 1
done; done
for i in 1 2; do
  DCA_LN_BWD_RG=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_rg_$i.log 2>&1 || exit 1
  DCA_LN_BWD_RG=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_old_$i.log 2>&1 || exit 1
done
