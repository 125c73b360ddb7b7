set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bnred2
mkdir -p $O
python -c "import determined_clone_amd.ops._C" || exit 1
for cfg in "4,0" "4,1" "8,0" "8,1" "4,0"; do
  DCA_BN_REDUCE_VAR=$cfg timeout -k 10 200 python tools/bench_bn.py --batch 1024 > "$O/bn_$cfg.txt" 2>&1 || exit 1
  echo "$cfg: $(tail -1 "$O/bn_$cfg.txt")"
done
