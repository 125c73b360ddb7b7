# round 5: stem weight-gradient MFMA kernel: numerics, standalone time vs MIOpen, in-step A/B
set -o pipefail
OUT=gpurun_out/r5w7
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem > $OUT/test.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_stem_s2d.py > $OUT/micro.txt 2>&1 || exit 1
for ab in 1 0 1 0; do
  DCA_STEM_WGRAD=$ab timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/b.log 2>&1 || exit 1
  echo "stem_wgrad=$ab $(tail -1 $OUT/b.log | cut -c1-90)" >> $OUT/ab.txt
done
