set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm7
mkdir -p $O
python -c "import determined_clone_amd.ops._C" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1
rc=$?; tail -3 $O/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_igemm.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v "amdgpu.ids" $O/bench.txt | grep -v '"k": 1'
