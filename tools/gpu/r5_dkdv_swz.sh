# round 5: dK/dV kernel (D64) with the swizzled unpadded layout (DCA_ATTN_DKDV_SWZ=1): numerics, A/B
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
DCA_ATTN_DKDV_SWZ=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash_attention or hf_models" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --only bwd > $OUT/bwd_base_$i.jsonl 2>>$OUT/err.txt || exit 1
  DCA_ATTN_DKDV_SWZ=1 timeout -k 10 120 python tools/bench_attn.py --only bwd > $OUT/bwd_swz_$i.jsonl 2>>$OUT/err.txt || exit 1
done
for i in 1 2; do
  DCA_ATTN_DKDV_SWZ=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_swz_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_base_$i.log 2>&1 || exit 1
done
