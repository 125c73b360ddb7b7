# round 5: attention -- numerics of the 64-rows-per-wave forward, A/B against the current forward,
# and PMC counters of both (one counter pass per run)
set -o pipefail
OUT=gpurun_out/r5j
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DCA_ATTN_FWD_W64=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "flash_attention or hf_models" > $OUT/pytest_w64.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/bench_attn.py --only fwd > $OUT/attn_base_$i.jsonl 2>>$OUT/attn.err || exit 1
  timeout -k 10 120 python tools/bench_attn.py --only fwd --noncausal --shapes "4,4096,8,128;8,2048,16,64" >> $OUT/attn_base_$i.jsonl 2>>$OUT/attn.err || exit 1
  DCA_ATTN_FWD_W64=1 timeout -k 10 120 python tools/bench_attn.py --only fwd > $OUT/attn_w64_$i.jsonl 2>>$OUT/attn.err || exit 1
  DCA_ATTN_FWD_W64=1 timeout -k 10 120 python tools/bench_attn.py --only fwd --noncausal --shapes "4,4096,8,128;8,2048,16,64" >> $OUT/attn_w64_$i.jsonl 2>>$OUT/attn.err || exit 1
done
timeout -k 10 120 python tools/bench_attn.py --only bwd > $OUT/attn_bwd.jsonl 2>>$OUT/attn.err || exit 1
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d $OUT/pmc1 -o run -- python tools/bench_attn.py --iters 3 > $OUT/pmc1.log 2>&1 || exit 1
DCA_ATTN_FWD_W64=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d $OUT/pmc1w -o run -- python tools/bench_attn.py --iters 3 --only fwd > $OUT/pmc1w.log 2>&1 || exit 1
