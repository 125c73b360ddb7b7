# round 6: GPT-2 weight-gradient side stream on a CU subset (DCA_WGRAD_CU_MASK=N/D) vs the whole chip
set -o pipefail
OUT=gpurun_out/r6cum
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "side or wgrad or linear" > $OUT/pytest_none.log 2>&1 || exit 1
DCA_WGRAD_CU_MASK=3/4 timeout -k 10 120 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "side or wgrad or linear" > $OUT/pytest_3of4.log 2>&1 || exit 1
for i in 1 2; do
  for m in none 7/8 3/4 1/2; do
    tag=$(echo $m | tr / o)
    if [ $m = none ]; then
      timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_${tag}_$i.log 2>&1 || exit 1
    else
      DCA_WGRAD_CU_MASK=$m timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_${tag}_$i.log 2>&1 || exit 1
    fi
  done
done
