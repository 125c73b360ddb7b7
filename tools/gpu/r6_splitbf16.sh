# round 6: split-K weight-gradient slices in bf16 vs fp32 -- isolated GEMM timing, kernel numerics, GPT-2 step A/B
set -o pipefail
OUT=gpurun_out/r6m
mkdir -p $OUT
timeout -k 10 200 python tools/probe_bmm_out.py > $OUT/bmm.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "splitk or linear_direct" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  DCA_SPLITK_BF16=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt_bf16_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt_f32_$i.log 2>&1 || exit 1
done
