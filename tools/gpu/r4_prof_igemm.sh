# rocprofv3 step breakdown of the ResNet-50 bench with and without the implicit-GEMM convs
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/r4prof
for v in 1 0; do
  cd /tmp && DCA_IGEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r4prof/ig$v -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/gpurun_out/r4prof/bench_ig$v.log 2>&1 || exit 1
  cd $ROOT && f=$(find gpurun_out/r4prof/ig$v -name 'run_kernel_trace.csv' | head -1) && \
  python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > gpurun_out/r4prof/breakdown_ig$v.txt && rm -f $f || exit 1
  head -30 gpurun_out/r4prof/breakdown_ig$v.txt
done
