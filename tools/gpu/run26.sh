set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r26_pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r26_pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/r26_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r26_smoke.txt 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r26_smoke.txt; exit 1; }
grep "smoke ok" gpurun_out/r26_smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r26_bench.txt 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r26_bench.txt; exit 1; }
tail -1 gpurun_out/r26_bench.txt | cut -c1-200
timeout -k 10 400 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/r26_gpt.txt 2>&1 || { echo "gpt bench failed"; tail -30 gpurun_out/r26_gpt.txt; exit 1; }
tail -1 gpurun_out/r26_gpt.txt | cut -c1-200
