set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
for b in 512 384 256 192; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --batch $b > gpurun_out/r22_bs$b.txt 2>&1 || { echo "bench bs=$b failed"; tail -20 gpurun_out/r22_bs$b.txt; exit 1; }
  echo "bs=$b $(tail -1 gpurun_out/r22_bs$b.txt | cut -c1-130)"
done
