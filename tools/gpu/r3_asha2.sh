set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3asha2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python tools/bench_asha.py --trace > $O/asha_$i.txt 2>&1 || exit $?
done
grep -h 'startup\|"metric"' $O/asha_*.txt | cut -c1-200
