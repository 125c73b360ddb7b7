# round 5: stem BN+ReLU+maxpool backward in quad form (one thread per 2x2 block): tests, in-step A/B, kernel times
set -o pipefail
OUT=gpurun_out/r5q3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "maxpool or stem" > $OUT/test.log 2>&1 || exit 1
for ab in 1 1; do
  DCA_BN_POOL_QUAD=$ab timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/b.log 2>&1 || exit 1
  echo "quad=$ab $(tail -1 $OUT/b.log | cut -c1-90)" >> $OUT/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 4 --warmup 3 > $OUT/prof.log 2>&1 || exit 1
