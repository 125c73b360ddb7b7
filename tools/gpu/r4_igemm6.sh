set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1
rc=$?; tail -3 $O/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_igemm.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v "amdgpu.ids" $O/bench.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_step.txt 2> $O/bench_step.err || { tail $O/bench_step.err; exit 1; }
tail -1 $O/bench_step.txt
DCA_IGEMM=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_noigemm.txt 2> $O/bench_noigemm.err || exit 1
tail -1 $O/bench_noigemm.txt
