#!/bin/bash
# end-of-session check on the final tree: full GPU tier, smoke, driver bench; then a same-box
# A/B of forcing every eligible 1x1 convolution onto the implicit GEMM with BN statistics
set -o pipefail
O=gpurun_out/r4close2
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
timeout -k 10 300 python bench.py > $O/bench_default_args.txt 2> $O/bench_default_args.err || exit $?
cut -c1-260 $O/bench_default_args.txt
for r in 1 2; do
  for v in auto 1; do
    DCA_IG1X1=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/b_$v.txt 2>/dev/null || exit 1
    echo "## IG1X1=$v round $r: $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d["value"], d["ms_per_step"])' $O/b_$v.txt)"
  done
done
