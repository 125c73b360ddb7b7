# round 5: stem space-to-depth kernel: bit-exact test, stem kernel time, in-step A/B (ResNet-50 bs 1024)
set -o pipefail
OUT=gpurun_out/r5c3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null

timeout -k 10 120 python tools/bench_stem_s2d.py > $OUT/micro.txt 2>&1 || exit 1
for ab in 1 0; do
  export DCA_STEM_KERNEL=$ab
  timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $OUT/bench_$ab.log 2>&1 || exit 1
  echo "stem_kernel=$ab $(tail -1 $OUT/bench_$ab.log)" >> $OUT/ab.txt
done
unset DCA_STEM_KERNEL
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python tools/bench_stem_s2d.py > $OUT/prof.log 2>&1 || exit 1
