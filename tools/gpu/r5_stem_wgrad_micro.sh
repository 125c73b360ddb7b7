# round 5: stem weight-gradient kernel numerics + standalone time
set -o pipefail
OUT=gpurun_out/r5w8
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k wgrad_kernel > $OUT/test.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_stem_s2d.py > $OUT/micro.txt 2>&1 || exit 1
