# side-stream weight gradients: numerics test + same-box A/B of the ResNet-50 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread -k "side_stream or pointwise" > gpurun_out/wg_pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/wg_bench_off.txt 2>&1 &&
DCA_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/wg_bench_on.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/wg_bench_off2.txt 2>&1 &&
DCA_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/wg_bench_on2.txt 2>&1
