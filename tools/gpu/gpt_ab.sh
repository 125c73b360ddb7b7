set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_gpt2.py tests/test_zero.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpt_pytest.txt 2>&1 &&
DCA_LINEAR_WGRAD_STREAM=0 timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/gpt_off.txt 2>&1 &&
DCA_LINEAR_WGRAD_STREAM=1 timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/gpt_on.txt 2>&1 &&
DCA_LINEAR_WGRAD_STREAM=0 timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/gpt_off2.txt 2>&1 &&
DCA_LINEAR_WGRAD_STREAM=1 timeout -k 10 300 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/gpt_on2.txt 2>&1
