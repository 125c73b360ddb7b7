# round 6: big-tile implicit GEMM, 3-deep ring -- numerics + isolated A/B (old 4-wave / 256x128 / 128x256) + step A/B
set -o pipefail
OUT=gpurun_out/r6c
mkdir -p $OUT
OLD=tools/bin/_C_igemm_old.so
V2=tools/bin/_C_igemm_v2.so
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1 || exit 1
DCA_OPS_SO=$V2 timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k igemm > $OUT/pytest_conv_v2.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm_v1.jsonl 2> $OUT/igemm_v1.err || exit 1
DCA_OPS_SO=$V2 timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm_v2.jsonl 2> $OUT/igemm_v2.err || exit 1
DCA_OPS_SO=$OLD timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm_old.jsonl 2> $OUT/igemm_old.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_v1_$i.log 2>&1 || exit 1
  DCA_OPS_SO=$V2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_v2_$i.log 2>&1 || exit 1
  DCA_OPS_SO=$OLD timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_old_$i.log 2>&1 || exit 1
done
