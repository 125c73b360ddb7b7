set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r20_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r20_pytest.txt; exit 1; }
tail -3 gpurun_out/r20_pytest.txt
timeout -k 10 300 python -u tools/bench_pointwise.py > gpurun_out/r20_pointwise.txt 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r20_pointwise.txt; exit 1; }
cat gpurun_out/r20_pointwise.txt | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r20_bench.txt 2>&1 || { echo "resnet bench failed"; tail -30 gpurun_out/r20_bench.txt; exit 1; }
tail -1 gpurun_out/r20_bench.txt | cut -c1-200
