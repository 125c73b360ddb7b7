# round 5: ResNet-50 step kernel traces with / without the stem convolution kernel (same box)
set -o pipefail
OUT=gpurun_out/r5c4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for ab in 1 0; do
  export DCA_STEM_KERNEL=$ab
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof$ab -o run -- python bench.py --steps 6 --warmup 3 > $OUT/bench$ab.log 2>&1 || exit 1
done
