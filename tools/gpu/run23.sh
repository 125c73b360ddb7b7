set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r23_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r23_pytest.txt; exit 1; }
tail -4 gpurun_out/r23_pytest.txt
for hg in 1 0; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --hip-graph $hg > gpurun_out/r23_bench_hg$hg.txt 2>&1 || { echo "bench hg=$hg failed"; tail -30 gpurun_out/r23_bench_hg$hg.txt; exit 1; }
  echo "hip_graph=$hg $(tail -1 gpurun_out/r23_bench_hg$hg.txt | cut -c1-140)"
done
