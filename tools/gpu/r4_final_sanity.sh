#!/bin/bash
# final tree sanity: full GPU tier, smoke, driver-default bench
set -o pipefail
O=gpurun_out/r4sanity
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
tail -2 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench.txt 2> $O/bench.err || exit $?
cut -c1-240 $O/bench.txt
