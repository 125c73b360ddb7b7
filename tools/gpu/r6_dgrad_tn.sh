# round 6: data-gradient GEMMs in the TN layout (transposed weight copy, DCA_DGRAD_TN=1) vs NN:
# isolated probe, TunableOp tuning of the new TN shapes (seeded with the shipped results, so only
# new shapes are timed), then GPT-2 and ResNet-50 step A/B on the merged results
set -o pipefail
OUT=gpurun_out/r6tn
mkdir -p $OUT
(while true; do date > $OUT/heartbeat; sleep 20; done) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python tools/probe_dgrad_tn.py > $OUT/probe_replay.txt 2>&1 || exit 1
cp determined_clone_amd/ops/tuned/gemm_gfx950.csv $OUT/tune.csv
DCA_DGRAD_TN=1 DCA_GEMM_TUNE=$OUT/tune.csv timeout -k 10 400 python tools/bench_gpt2.py --steps 2 --warmup 1 > $OUT/tune_gpt2.log 2>&1 || exit 1
DCA_DGRAD_TN=1 DCA_GEMM_TUNE=$OUT/tune.csv timeout -k 10 400 python bench.py --steps 2 --warmup 1 > $OUT/tune_rn.log 2>&1 || exit 1
DCA_GEMM_TUNE=$OUT/tune.csv timeout -k 10 300 python tools/probe_dgrad_tn.py > $OUT/probe_tune.txt 2>&1 || exit 1
cp $OUT/tune.csv determined_clone_amd/ops/tuned/gemm_gfx950.csv
timeout -k 10 300 python tools/probe_dgrad_tn.py > $OUT/probe_tuned.txt 2>&1 || exit 1
DCA_DGRAD_TN=1 timeout -k 10 200 python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_tn.log 2>&1 || exit 1
for i in 1 2; do
  for t in 0 1; do
    DCA_DGRAD_TN=$t timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_tn${t}_$i.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for t in 0 1; do
    DCA_DGRAD_TN=$t timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_tn${t}_$i.log 2>&1 || exit 1
  done
done
