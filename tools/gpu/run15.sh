set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/r15_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r15_pytest.txt; exit 1; }
tail -2 gpurun_out/r15_pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r15_smoke.txt 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r15_smoke.txt; exit 1; }
tail -2 gpurun_out/r15_smoke.txt
timeout -k 10 1000 python tools/bench_asha.py --slots-per-gpu 8 --max-trials 32 --max-concurrent 8 --epochs 4 --records-per-epoch 6400 --timeout 900 > gpurun_out/r15_asha.txt 2> gpurun_out/r15_asha_err.txt
echo "asha rc=$?"
tail -1 gpurun_out/r15_asha.txt
