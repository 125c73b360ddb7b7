set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c
mkdir -p $O
export DCA_CONV_DEBUG=1
for i in 1 2 3 4; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit $?
done
grep -h "metric\|step_ms" $O/bench_*.log | cut -c1-400
