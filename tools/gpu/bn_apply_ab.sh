# BN apply passes: rows in flight per lane x workgroup cap (DCA_BN_APPLY="U,max_blocks"), bs512 bench
set -o pipefail
mkdir -p gpurun_out/bn_apply
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "bn or batchnorm" > gpurun_out/bn_apply/tests.txt 2>&1 || exit 1
for v in 4,2048 8,2048 2,2048 4,4096 8,1024 4,2048; do
  DCA_BN_APPLY=$v timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bn_apply/b_$v.$RANDOM.txt 2>&1 || exit 1
done
