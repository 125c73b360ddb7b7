# round 5: attention DMA ring defaults (fwd all, dQ all, dK/dV D128) vs register staging; GPT-2 A/B;
# PMC pass of the new defaults
set -o pipefail
OUT=gpurun_out/r5o
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash_attention or hf_models" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  DCA_ATTN_FWD_DMA=0 DCA_ATTN_BWD_DMA=0 timeout -k 10 120 python tools/bench_attn.py > $OUT/attn_reg_$i.jsonl 2>>$OUT/err.txt || exit 1
  timeout -k 10 120 python tools/bench_attn.py > $OUT/attn_dma_$i.jsonl 2>>$OUT/err.txt || exit 1
done
DCA_ATTN_FWD_DMA=0 DCA_ATTN_BWD_DMA=0 timeout -k 10 120 python tools/bench_attn.py --noncausal --shapes "4,4096,8,128;8,2048,16,64" > $OUT/attn_reg_nc.jsonl 2>>$OUT/err.txt || exit 1
timeout -k 10 120 python tools/bench_attn.py --noncausal --shapes "4,4096,8,128;8,2048,16,64" > $OUT/attn_dma_nc.jsonl 2>>$OUT/err.txt || exit 1
for i in 1 2; do
  timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_dma_$i.log 2>&1 || exit 1
  DCA_ATTN_FWD_DMA=0 DCA_ATTN_BWD_DMA=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt_reg_$i.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d $OUT/pmc -o run -- python tools/bench_attn.py --iters 3 > $OUT/pmc.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d $OUT/pmc_lds -o run -- python tools/bench_attn.py --iters 3 > $OUT/pmc_lds.log 2>&1 || exit 1
