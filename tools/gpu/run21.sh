set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r21_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r21_pytest.txt; exit 1; }
tail -1 gpurun_out/r21_pytest.txt
for bm in 64 128 256; do
for wg in 512 2048; do
DCA_PW_BM=$bm DCA_PW_WG_BLOCKS=$wg timeout -k 10 300 python -u tools/bench_pointwise.py > gpurun_out/r21_pw_${bm}_${wg}.txt 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r21_pw_${bm}_${wg}.txt; exit 1; }
echo "bm=$bm wg=$wg $(tail -1 gpurun_out/r21_pw_${bm}_${wg}.txt)"
done
done
