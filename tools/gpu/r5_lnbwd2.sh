# round 5: LN backward (row-group kernel, one column-reduce launch) -- numerics, micro-benchmark,
# GPT-2 A/B of the out-projection bias gradient reduced in the LN backward (fused) vs separate
set -o pipefail
OUT=gpurun_out/r5h
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py \
  > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_ln_bwd.py > $OUT/micro.jsonl 2>$OUT/micro.err || exit 1
for i in 1 2; do
  DCA_FUSE_LN_BIAS_GRAD=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_fused_$i.log 2>&1 || exit 1
  DCA_FUSE_LN_BIAS_GRAD=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_sep_$i.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python tools/bench_gpt2.py --steps 4 --warmup 3 > $OUT/prof_bench.log 2>&1 || exit 1
