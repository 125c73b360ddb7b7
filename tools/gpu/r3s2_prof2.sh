# GPT-2 step breakdown after the attention work + SD UNet bench and breakdown
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/s2prof2
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/gprof -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 4 --warmup 3 > $O/gpt2.log 2>&1 || exit $?
cd $ROOT && f=$(find $O/gprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 9 adam_kernel "" attn_ > $O/gpt2_breakdown.txt && rm -f $f || exit $?
timeout -k 10 300 python3 tools/bench_diffusion.py > $O/sd.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/sprof -o run --output-format csv -- python3 $ROOT/tools/bench_diffusion.py --steps 4 --warmup 3 > $O/sd_prof.log 2>&1 || exit $?
cd $ROOT && f=$(find $O/sprof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 3 1 adam_kernel "" attn_ > $O/sd_breakdown.txt && rm -f $f
grep -h images_per_s $O/sd.txt
