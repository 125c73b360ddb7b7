set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm1
mkdir -p $O
timeout -k 10 120 python tools/bench_igemm.py --check-only > $O/check.txt 2>&1 || { cat $O/check.txt; exit 1; }
cat $O/check.txt
timeout -k 10 300 python tools/bench_igemm.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
for cfg in "2,100000000" "1,100000000" "4,100000000"; do
  DCA_BN_APPLY=$cfg timeout -k 10 200 python tools/bench_bn.py --batch 1024 > $O/bn_$cfg.txt 2>&1 || exit 1
done
timeout -k 10 200 python tools/bench_bn.py --batch 1024 > $O/bn_default.txt 2>&1
