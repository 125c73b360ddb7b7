set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_transformer_ops_gpu.py tests/test_ops_gpu.py tests/test_gpt2.py tests/test_zero.py -q -m gpu -x -p no:cacheprovider > gpurun_out/r18_pytest.txt 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/r18_pytest.txt; exit 1; }
tail -2 gpurun_out/r18_pytest.txt
for dg in 1 0; do
  DCA_DIRECT_GRAD=$dg timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r18_resnet_dg$dg.txt 2>&1 || { echo "resnet bench failed"; tail -30 gpurun_out/r18_resnet_dg$dg.txt; exit 1; }
  echo "resnet DCA_DIRECT_GRAD=$dg: $(tail -1 gpurun_out/r18_resnet_dg$dg.txt | cut -c1-140)"
done
for dg in 0 1; do
  DCA_DIRECT_GRAD=$dg timeout -k 10 400 python tools/bench_gpt2.py --micro 16 --steps 20 --warmup 5 > gpurun_out/r18_gpt_dg$dg.txt 2>&1 || { echo "gpt bench failed"; tail -30 gpurun_out/r18_gpt_dg$dg.txt; exit 1; }
  echo "gpt DCA_DIRECT_GRAD=$dg: $(tail -1 gpurun_out/r18_gpt_dg$dg.txt | cut -c1-160)"
done
