set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_diffusion_gpu.py tests/test_groupnorm_gpu.py tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sd2_pytest.txt 2>&1 &&
timeout -k 10 400 python tools/bench_diffusion.py --batch 8 --res 512 --steps 8 --warmup 3 > gpurun_out/sd2_bench.txt 2>&1 &&
DCA_WGRAD_STREAM=0 DCA_LINEAR_WGRAD_STREAM=0 timeout -k 10 400 python tools/bench_diffusion.py --batch 8 --res 512 --steps 8 --warmup 3 > gpurun_out/sd2_bench_noside.txt 2>&1
