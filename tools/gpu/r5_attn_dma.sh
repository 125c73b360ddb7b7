# round 5: attention forward with the direct-to-LDS K/V ring (DCA_ATTN_FWD_DMA=1): numerics, then A/B
set -o pipefail
OUT=gpurun_out/r5m
mkdir -p $OUT
DCA_ATTN_FWD_DMA=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash_attention or hf_models" > $OUT/pytest_dma.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" > $OUT/base_$i.jsonl 2>>$OUT/err.txt || exit 1
  DCA_ATTN_FWD_DMA=1 timeout -k 10 120 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" > $OUT/dma_$i.jsonl 2>>$OUT/err.txt || exit 1
done
timeout -k 10 120 python tools/bench_attn.py --only fwd --noncausal --shapes "4,4096,8,128;8,2048,16,64" > $OUT/base_nc.jsonl 2>>$OUT/err.txt || exit 1
DCA_ATTN_FWD_DMA=1 timeout -k 10 120 python tools/bench_attn.py --only fwd --noncausal --shapes "4,4096,8,128;8,2048,16,64" > $OUT/dma_nc.jsonl 2>>$OUT/err.txt || exit 1
