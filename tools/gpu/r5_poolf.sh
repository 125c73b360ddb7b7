# round 5: stem BN+ReLU+max-pool FORWARD in quad form (2x2 pooled outputs per thread): tests, kernel time, in-step A/B
set -o pipefail
OUT=gpurun_out/r5pf
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_conv_gpu.py -k "maxpool or stem" > $OUT/test.log 2>&1 || exit 1
for ab in 1 0; do
  DCA_BN_POOL_FWD_QUAD=$ab timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$ab -o run -- python bench.py --steps 4 --warmup 3 > $OUT/prof$ab.log 2>&1 || exit 1
done
for ab in 1 0 1 0; do
  DCA_BN_POOL_FWD_QUAD=$ab timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/b.log 2>&1 || exit 1
  echo "pool_fwd_quad=$ab $(tail -1 $OUT/b.log | cut -c1-90)" >> $OUT/ab.txt
done
