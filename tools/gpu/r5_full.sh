# round 5: full GPU tier + smoke + bench (the driver's round-end sequence) on the current tree
set -o pipefail
OUT=gpurun_out/r5f4
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gpt2.py --steps 20 --warmup 5 > $OUT/gpt2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 4 --warmup 3 > $OUT/prof.log 2>&1 || exit 1
