# round 5: hipBLASLt epilogue MLP (DCA_LT_MLP=1): numerics, then GPT-2 A/B
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "mlp_gelu" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  DCA_LT_MLP=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_lt_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_base_$i.log 2>&1 || exit 1
done
