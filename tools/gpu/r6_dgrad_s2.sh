# round 6: 3x3 stride-2 data gradient as parity-class implicit GEMMs -- numerics, isolated timing vs MIOpen, step A/B
set -o pipefail
OUT=gpurun_out/r6r
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm.jsonl 2> $OUT/igemm.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$i.log 2>&1 || exit 1
  DCA_IGEMM_DGRAD_S2=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_base_$i.log 2>&1 || exit 1
done
