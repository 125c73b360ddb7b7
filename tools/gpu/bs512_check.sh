# default bench (bs 512 per GPU) from the in-tree MIOpen DB: wall time incl. warmup, then a kernel trace
set -o pipefail
mkdir -p gpurun_out
( time timeout -k 10 500 python bench.py ) > gpurun_out/bs512_default.txt 2>&1 &&
bash tools/gpu/prof_resnet.sh
