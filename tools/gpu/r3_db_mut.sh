set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
export DCA_CONV_DEBUG=1
cp -a tools/miopen /tmp/miopen_pristine
ls -la --time-style=full-iso tools/miopen/db tools/miopen/cache > $O/ls_before.txt
ls -la ~/.cache/miopen ~/.config/miopen > $O/home_before.txt 2>&1 || true
# run 1: as shipped
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_1.log 2>&1 || exit $?
ls -la --time-style=full-iso tools/miopen/db tools/miopen/cache > $O/ls_after1.txt
ls -laR ~/.cache/miopen ~/.config/miopen > $O/home_after1.txt 2>&1 || true
mkdir -p $O/db_after1 && cp -a tools/miopen/db/* $O/db_after1/ 2>/dev/null
# run 2: restore the pristine DB first
rm -rf tools/miopen && cp -a /tmp/miopen_pristine tools/miopen
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_2.log 2>&1 || exit $?
# run 3: do not restore (mutated by run 2)
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_3.log 2>&1 || exit $?
ls -laR ~/.cache/miopen ~/.config/miopen > $O/home_after3.txt 2>&1 || true
# run 4: restore DB and wipe home caches
rm -rf tools/miopen && cp -a /tmp/miopen_pristine tools/miopen
rm -rf ~/.cache/miopen ~/.config/miopen
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_4.log 2>&1 || exit $?
grep -h metric $O/bench_*.log | cut -c1-120
