set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_transformer_ops_gpu.py -q -m gpu > gpurun_out/r4_pytest.txt 2>&1; rc=$?
tail -40 gpurun_out/r4_pytest.txt
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -q "Fatal\|core dumped\|Aborted\|Segmentation" gpurun_out/r4_pytest.txt && exit 1; fi
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/r4_bench_ops.txt 2>&1; echo "bench_ops rc=$?"
cat gpurun_out/r4_bench_ops.txt | tail -20
