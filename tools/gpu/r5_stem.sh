# round 5: stem space-to-depth kernel: bit-exact test, stem kernel time, in-step A/B (ResNet-50 bs 1024)
set -o pipefail
OUT=gpurun_out/r5s2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k stem > $OUT/test.log 2>&1 || exit 1
timeout -k 10 120 python tools/bench_stem_s2d.py > $OUT/micro.txt 2>&1 || exit 1
for ab in 1 0 1 0; do
  DCA_STEM_S2D_KERNEL=$ab timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/bench_$ab.log 2>&1 || exit 1
  echo "kernel=$ab $(tail -1 $OUT/bench_$ab.log)" >> $OUT/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/bench_stem_s2d.py > $OUT/prof.log 2>&1 || exit 1
