# round-4 closing check: full GPU tier, smoke, driver bench, GPT-2 bench, attention throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4final
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc  # any failed GPU test ends the check
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.txt 2> $O/bench.err || exit $?
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt2.txt 2>&1 || exit $?
timeout -k 10 200 python tools/bench_attn.py > $O/attn.txt 2>&1 || exit $?
grep -h '"metric"' $O/bench.txt $O/gpt2.txt | cut -c1-300; tail -2 $O/smoke.txt; grep -h '"pass"' $O/attn.txt | cut -c1-130
