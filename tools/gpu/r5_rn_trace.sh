# round 5: ResNet-50 step kernel trace (csv) to attribute the main-stream copies
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python bench.py --steps 4 --warmup 3 > $OUT/bench.log 2>&1 || exit 1
