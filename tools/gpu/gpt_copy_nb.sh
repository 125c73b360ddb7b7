# GPT-2-medium ZeRO-2 micro 32: which kernels surround the __amd_rocclr_copyBuffer launches (8.8% of GPU time)
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/gptnb
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/gptnb/prof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --micro 32 --steps 4 --warmup 3 > $ROOT/gpurun_out/gptnb/bench.log 2>&1 && \
cd $ROOT && f=$(find gpurun_out/gptnb/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 9 adam_kernel __amd_rocclr_copyBuffer > gpurun_out/gptnb/breakdown.txt && \
rm -f $f
