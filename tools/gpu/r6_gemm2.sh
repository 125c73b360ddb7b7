# round 6: GPT-2 step A/B with the MLP backward on the 256x256 GEMM's dGELU epilogue
set -o pipefail
OUT=gpurun_out/r6i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "gelu_linear or dgelu" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  DCA_FUSE_MLP_DGELU=1 timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_fused_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_base_$i.log 2>&1 || exit 1
done
