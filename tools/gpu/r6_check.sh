# round 6 closing check on the final tree: full GPU tier, smoke, bench.py, GPT-2, attention, kernel stats
set -o pipefail
OUT=gpurun_out/r6check
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_attn.py > $OUT/attn.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 3 > $OUT/prof.log 2>&1 || exit 1
