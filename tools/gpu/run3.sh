set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -x -q -m gpu > gpurun_out/r3_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r3_pytest.txt; exit 1; }
( time timeout -k 10 600 python bench.py --steps 30 --warmup 10 ) > gpurun_out/r3_bench1.txt 2>&1 || { echo "bench1 failed"; tail -20 gpurun_out/r3_bench1.txt; exit 1; }
mkdir -p gpurun_out/miopen && cp -r tools/miopen/db tools/miopen/cache gpurun_out/miopen/ 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof3 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 3 > $ROOT/gpurun_out/r3_prof_stdout.txt 2>&1
echo "prof rc=$?"
