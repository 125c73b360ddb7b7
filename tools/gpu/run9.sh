set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_transformer_ops_gpu.py -q -m gpu -x -k attention 2>&1 | tee gpurun_out/r9_pytest.txt | tail -30
timeout -k 10 300 python tools/bench_ops.py 2>&1 | tee gpurun_out/r9_bench_ops.txt
