set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/sdprof -o run --output-format csv -- python3 $ROOT/tools/bench_diffusion.py --batch 8 --res 512 --steps 4 --warmup 2 > $ROOT/gpurun_out/sdprof_stdout.txt 2>&1 && \
cd $ROOT && f=$(find gpurun_out/sdprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 1 adam_kernel > gpurun_out/sd_breakdown.txt && rm -f $f
