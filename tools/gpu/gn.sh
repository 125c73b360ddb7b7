set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_groupnorm_gpu.py tests/test_diffusion_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gn_pytest.txt 2>&1 &&
timeout -k 10 400 python tools/bench_diffusion.py --batch 8 --res 512 --steps 8 --warmup 3 > gpurun_out/gn_bench_fused.txt 2>&1 &&
DCA_GN_TORCH=1 timeout -k 10 400 python tools/bench_diffusion.py --batch 8 --res 512 --steps 8 --warmup 3 > gpurun_out/gn_bench_torch.txt 2>&1
