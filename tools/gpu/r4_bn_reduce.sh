set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bnred
mkdir -p $O
for cfg in "32768,256,2048" "16384,256,8192,1048576" "8192,256,16384,2097152" "4096,256,32768,4194304" "32768,256,2048"; do
  DCA_BN_REDUCE=$cfg timeout -k 10 200 python tools/bench_bn.py --batch 1024 > "$O/bn_$cfg.txt" 2>&1 || exit 1
  echo "$cfg: $(tail -1 "$O/bn_$cfg.txt")"
done
timeout -k 10 400 python tools/bench_igemm.py > $O/igemm_1x1.txt 2>&1 || { tail $O/igemm_1x1.txt; exit 1; }
grep '"k": 1\|per_step' $O/igemm_1x1.txt
