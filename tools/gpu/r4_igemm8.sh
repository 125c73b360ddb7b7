set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm8
mkdir -p $O
python -c "import determined_clone_amd.ops._C" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1
rc=$?; tail -3 $O/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_igemm.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
tail -1 $O/bench.txt
for bm in 256; do DCA_IGEMM_BM=$bm timeout -k 10 400 python tools/bench_igemm.py > $O/bench_bm$bm.txt 2>&1 || exit 1; echo "bm=$bm $(tail -1 $O/bench_bm$bm.txt)"; done
DCA_IGEMM_STAGES=3 timeout -k 10 400 python tools/bench_igemm.py > $O/bench_s3.txt 2>&1 || exit 1; echo "stages=3 $(tail -1 $O/bench_s3.txt)"
