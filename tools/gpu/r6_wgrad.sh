# round 6: implicit-GEMM weight gradient with incremental loader state -- numerics, isolated timing,
# re-decided per-shape choices (timed inside the bench process), step A/B against the shipped choices
set -o pipefail
OUT=gpurun_out/r6d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm.jsonl 2> $OUT/igemm.err || exit 1
DCA_CONV_CHOICES=0 DCA_CONV_DUMP=$OUT/choices.json DCA_CONV_DEBUG=1 timeout -k 10 400 python bench.py --steps 10 --warmup 5 > $OUT/bench_retime.log 2>&1 || exit 1
for i in 1 2; do
  DCA_CONV_CHOICES=$OUT/choices.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_shipped_$i.log 2>&1 || exit 1
done
