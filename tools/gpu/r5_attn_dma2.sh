# round 5: forward DMA ring (now default, unified swizzle) + backward DMA ring (DCA_ATTN_BWD_DMA=1):
# numerics, then A/B
set -o pipefail
OUT=gpurun_out/r5n
mkdir -p $OUT
DCA_ATTN_BWD_DMA=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash_attention or hf_models" > $OUT/pytest_dma.log 2>&1 || exit 1
for i in 1 2; do
  DCA_ATTN_FWD_DMA=0 timeout -k 10 120 python tools/bench_attn.py --only fwd > $OUT/fwd_reg_$i.jsonl 2>>$OUT/err.txt || exit 1
  timeout -k 10 120 python tools/bench_attn.py --only fwd > $OUT/fwd_dma_$i.jsonl 2>>$OUT/err.txt || exit 1
  timeout -k 10 120 python tools/bench_attn.py --only bwd > $OUT/bwd_reg_$i.jsonl 2>>$OUT/err.txt || exit 1
  DCA_ATTN_BWD_DMA=1 timeout -k 10 120 python tools/bench_attn.py --only bwd > $OUT/bwd_dma_$i.jsonl 2>>$OUT/err.txt || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DCA_ATTN_BWD_DMA=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/bench_attn.py --iters 5 > $OUT/prof.log 2>&1 || exit 1
