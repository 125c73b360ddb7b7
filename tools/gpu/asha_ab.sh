set -o pipefail
mkdir -p gpurun_out
DET_ZYGOTE=0 timeout -k 10 400 python tools/bench_asha.py > gpurun_out/asha_nozyg.txt 2>&1 &&
DET_ZYGOTE=1 timeout -k 10 400 python tools/bench_asha.py > gpurun_out/asha_zyg.txt 2>&1
