set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q -m gpu -x -p no:cacheprovider > gpurun_out/r16_pytest.txt 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r16_pytest.txt; exit 1; }
tail -2 gpurun_out/r16_pytest.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r16_bench.txt 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r16_bench.txt; exit 1; }
tail -1 gpurun_out/r16_bench.txt
for cfg in default 65536,256,1024 32768,512,2048 16384,1024,2048 16384,1024,4096 8192,2048,4096; do
  if [ $cfg = default ]; then unset DCA_BN_REDUCE; else export DCA_BN_REDUCE=$cfg; fi
  timeout -k 10 120 python tools/bench_bn.py >> gpurun_out/r16_bn_sweep.txt 2>&1 || { echo "bench_bn failed"; tail -20 gpurun_out/r16_bn_sweep.txt; exit 1; }
done
unset DCA_BN_REDUCE
grep -E "DCA_BN|weighted" gpurun_out/r16_bn_sweep.txt
