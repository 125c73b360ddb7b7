set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/benchab
mkdir -p $O
python -c "import determined_clone_amd.ops._C" || exit 1
for v in 1 0 1; do
  DCA_IGEMM=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_ig$v.txt 2> $O/bench_ig$v.err || { tail $O/bench_ig$v.err; exit 1; }
  echo "DCA_IGEMM=$v $(grep -o '"value": [0-9.]*' $O/bench_ig$v.txt)"
done
