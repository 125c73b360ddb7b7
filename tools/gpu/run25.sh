set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r25_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r25_pytest.txt; exit 1; }
tail -5 gpurun_out/r25_pytest.txt
timeout -k 10 300 python -u tools/bench_graph_step.py > gpurun_out/r25_graph_bench.txt 2>&1 || { echo "graph bench failed"; tail -30 gpurun_out/r25_graph_bench.txt; exit 1; }
grep speedup gpurun_out/r25_graph_bench.txt
