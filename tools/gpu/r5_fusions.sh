# round 5: GPU tests for the fused BN backward statistics (conv2 dgrad epilogue) and the LN-backward
# out-projection bias gradient, then same-box A/Bs (ResNet-50 bench, GPT-2 bench)
set -o pipefail
OUT=gpurun_out/r5f
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
[ -n "$SKIP_CONV_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_conv_gpu.py tests/test_ops_gpu.py -k "dgrad_bn or bn1_backward or bn_act or dual" \
  > $OUT/pytest_conv.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_gpt2.py \
  > $OUT/pytest_tr.log 2>&1 || exit 1
for i in 1 2; do
  DCA_FUSE_BN_BWD_STATS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/rn_fused_$i.log 2>&1 || exit 1
  DCA_FUSE_BN_BWD_STATS=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/rn_sep_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  DCA_FUSE_LN_BIAS_GRAD=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_fused_$i.log 2>&1 || exit 1
  DCA_FUSE_LN_BIAS_GRAD=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_sep_$i.log 2>&1 || exit 1
done
