set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_transformer_ops_gpu.py tests/test_gpt2.py -q -m gpu -x 2>&1 | tee gpurun_out/r10_pytest.txt | tail -15
timeout -k 10 300 python tools/bench_ops.py 2>&1 | tee gpurun_out/r10_bench_ops.txt
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 16 2>&1 | tee gpurun_out/r10_gpt2_m16.txt
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 8 2>&1 | tee gpurun_out/r10_gpt2_m8.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof10 -o run --output-format csv -- python3 $ROOT/tools/bench_gpt2.py --steps 4 --warmup 2 > $ROOT/gpurun_out/r10_prof_stdout.txt 2>&1
echo "prof rc=$?"
