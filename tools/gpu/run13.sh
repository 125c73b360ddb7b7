set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu -x > gpurun_out/r13_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r13_pytest.txt; exit 1; }
tail -2 gpurun_out/r13_pytest.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 10 2>&1 | tee gpurun_out/r13_bench_shipped.txt | tail -1
MIOPEN_USER_DB_PATH=$ROOT/tools/miopen_tuned/db MIOPEN_CUSTOM_CACHE_DIR=$ROOT/tools/miopen_tuned/cache timeout -k 10 300 python bench.py --steps 30 --warmup 10 2>&1 | tee gpurun_out/r13_bench_tuned.txt | tail -1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 2>&1 | tee gpurun_out/r13_bench_shipped2.txt | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof13 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 3 > $ROOT/gpurun_out/r13_prof_stdout.txt 2>&1
echo "prof rc=$?"
