# attention kernels after the uniform-branch / preload / LSE-vector changes: numerics + throughput + GPT-2 e2e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "attention or attn or flash or transformer or gpt" > gpurun_out/attn_tests.txt 2>&1 &&
timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn_bench.txt 2>&1 &&
timeout -k 10 400 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/attn_gpt2.txt 2>&1
