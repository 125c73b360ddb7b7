# ResNet-50 bs1024 step breakdown + kernel stats with this session's defaults
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/s2prof3
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rprof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $O/resnet.log 2>&1 || exit $?
cd $ROOT && f=$(find $O/rprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > $O/resnet_breakdown.txt && s=$(find $O/rprof -name 'run_kernel_stats.csv' | head -1) && head -40 $s | cut -c1-250 > $O/resnet_kernel_stats_head.csv && rm -f $f
head -14 $O/resnet_breakdown.txt
