set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r19_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r19_pytest.txt; exit 1; }
tail -4 gpurun_out/r19_pytest.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof19 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 3 > $ROOT/gpurun_out/r19_prof_stdout.txt 2>&1
echo "prof rc=$?"
