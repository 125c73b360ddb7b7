# round-4 first GPU check: HBM streaming ceilings, full GPU tier, driver bench (self-launch path)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4start
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 120 tools/bin/hbm_bw 1024 > $O/hbm_bw.txt 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.txt 2> $O/bench.err || exit $?
tail -1 $O/bench.txt
