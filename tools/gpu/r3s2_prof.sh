# round-3 session-2 baseline: wgrad side-stream noise floor, attention kernels, GPT-2 + ResNet-50 step breakdowns
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/s2prof
mkdir -p $O
timeout -k 10 120 python3 tools/dbg/wgrad_noise.py > $O/wgrad_noise.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_attn.py > $O/attn.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gprof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 4 --warmup 3 > $O/gpt2.log 2>&1 || exit $?
cd $ROOT && f=$(find $O/gprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 9 adam_kernel "" attn_ > $O/gpt2_breakdown.txt && rm -f $f || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rprof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $O/resnet.log 2>&1 || exit $?
cd $ROOT && f=$(find $O/rprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > $O/resnet_breakdown.txt && rm -f $f
