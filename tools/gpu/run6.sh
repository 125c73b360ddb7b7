set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 2>&1 | tee gpurun_out/r6_gpt2.txt
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 16 2>&1 | tee gpurun_out/r6_gpt2_m16.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof6 -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 4 --warmup 2 > $ROOT/gpurun_out/r6_prof_stdout.txt 2>&1
echo "prof rc=$?"
