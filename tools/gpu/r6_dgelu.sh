# round 6: fused MLP projection + dGELU backward (GPT-2) and the incremental-state implicit-GEMM
# weight gradient (ResNet-50): numerics, GPT-2 step A/B, igemm timing, re-decided conv choices, ResNet A/B
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "dgelu or gelu_linear or bias_gelu or linear_direct" > $OUT/pytest_tr.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_fused_$i.log 2>&1 || exit 1
  DCA_FUSE_MLP_DGELU=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_unfused_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/bench_igemm.py --batch 1024 > $OUT/igemm.jsonl 2> $OUT/igemm.err || exit 1
DCA_CONV_CHOICES=0 DCA_CONV_DUMP=$OUT/choices.json DCA_CONV_DEBUG=1 timeout -k 10 400 python bench.py --steps 10 --warmup 5 > $OUT/bench_retime.log 2>&1 || exit 1
for i in 1 2; do
  DCA_CONV_CHOICES=$OUT/choices.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_shipped_$i.log 2>&1 || exit 1
done
