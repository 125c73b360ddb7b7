# runtime environment A/B on the ResNet-50 bench: kernarg placement, MIOpen find mode
set -o pipefail
mkdir -p gpurun_out
S="--steps 20 --warmup 10"
( time timeout -k 10 300 python bench.py $S ) > gpurun_out/env_base.txt 2>&1 &&
( time HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py $S ) > gpurun_out/env_kernarg.txt 2>&1 &&
( time MIOPEN_FIND_MODE=1 timeout -k 10 600 python bench.py $S ) > gpurun_out/env_findnormal.txt 2>&1 &&
( time timeout -k 10 300 python bench.py $S ) > gpurun_out/env_base2.txt 2>&1
