# round 5: MIOpen stem convolution on the 16-channel S2D tensor (faster weight gradient) -- tests + in-step A/B
set -o pipefail
OUT=gpurun_out/r5s16
mkdir -p $OUT
DCA_STEM_S2D16=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem > $OUT/test.log 2>&1 || exit 1
for ab in 1 0 1 0; do
  DCA_STEM_S2D16=$ab timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/b.log 2>&1 || exit 1
  echo "s2d16=$ab $(tail -1 $OUT/b.log | cut -c1-90)" >> $OUT/ab.txt
done
