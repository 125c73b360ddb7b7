set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r2_smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
( time timeout -k 10 600 python bench.py --steps 30 --warmup 10 ) > gpurun_out/r2_bench1.txt 2>&1 || { echo "bench1 failed"; exit 1; }
du -sh tools/miopen/db tools/miopen/cache > gpurun_out/r2_miopen_sizes.txt 2>&1
( time timeout -k 10 600 python bench.py --steps 30 --warmup 10 ) > gpurun_out/r2_bench2.txt 2>&1 || { echo "bench2 failed"; exit 1; }
mkdir -p gpurun_out/miopen && cp -r tools/miopen/db gpurun_out/miopen/ 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof2 -o run --output-format csv -- python3 $ROOT/bench.py --steps 5 --warmup 3 > $ROOT/gpurun_out/r2_prof_stdout.txt 2>&1
echo "prof rc=$?"
