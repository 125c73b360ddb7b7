set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_conv1x1.py 2>&1 | tee gpurun_out/r8_conv1x1.txt
timeout -k 10 300 python -m pytest tests/test_transformer_ops_gpu.py -q -m gpu -k "layer_norm or bias_gelu" 2>&1 | tail -3
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 16 2>&1 | tee gpurun_out/r8_gpt2_m16.txt
