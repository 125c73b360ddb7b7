# round 6: 8-wave big-tile implicit GEMM -- numerics, isolated A/B vs the 4-wave kernel, step A/B
set -o pipefail
OUT=gpurun_out/r6b
mkdir -p $OUT
OLD=tools/bin/_C_igemm_old.so
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm_new.jsonl 2> $OUT/igemm_new.err || exit 1
DCA_OPS_SO=$OLD timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm_old.jsonl 2> $OUT/igemm_old.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$i.log 2>&1 || exit 1
  DCA_OPS_SO=$OLD timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_old_$i.log 2>&1 || exit 1
done
