# space-to-depth stem: MIOpen find for its shapes (DB copied back), numerics, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3stem
mkdir -p $O/db
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python tools/bench_conv3x3.py --find --only-stem > $O/stem_find.txt 2>&1 || exit $?
cp -a determined_clone_amd/ops/tuned/miopen/db/. $O/db/ && cp -a determined_clone_amd/ops/tuned/miopen/cache/. $O/db/
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem > $O/pytest.log 2>&1 || exit $?
DCA_STEM_S2D=0 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_plain.txt 2>&1 || exit $?
DCA_STEM_S2D=1 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_s2d.txt 2>&1 || exit $?
DCA_STEM_S2D=0 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_plain2.txt 2>&1 || exit $?
DCA_STEM_S2D=1 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench_s2d2.txt 2>&1 || exit $?
tail -1 $O/pytest.log; grep -h -o '"value": [0-9.]*' $O/bench_*.txt
