# BN finalize rework: numerics, then a kernel trace of the bs512 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "bn or batchnorm or resnet or conv" > gpurun_out/bn_fin_tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bn_fin_bench.txt 2>&1 &&
bash tools/gpu/prof_resnet.sh
