# round 6: attention forward with pre-scaled Q and score-origin accumulators -- numerics, then A/B vs the previous kernel
set -o pipefail
OUT=gpurun_out/r6k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python tools/bench_attn.py > $OUT/new_$i.txt 2>&1 || exit 1
  DCA_OPS_SO=tools/bin/_C_attn_old.so timeout -k 10 200 python tools/bench_attn.py > $OUT/old_$i.txt 2>&1 || exit 1
done
