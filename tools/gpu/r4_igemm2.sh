set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm2
mkdir -p $O
timeout -k 10 120 python tools/bench_igemm.py --check-only > $O/check.txt 2>&1 || { cat $O/check.txt; exit 1; }
cat $O/check.txt
timeout -k 10 300 python tools/bench_igemm.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
DCA_IGEMM_BM=128 timeout -k 10 300 python tools/bench_igemm.py > $O/bench_bm128.txt 2>&1 || { tail $O/bench_bm128.txt; exit 1; }
cat $O/bench_bm128.txt
timeout -k 10 200 python tools/bench_bn.py --batch 1024 > $O/bn_new_default.txt 2>&1
tail -1 $O/bn_new_default.txt
