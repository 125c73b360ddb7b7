# A/B: training step on a high-priority stream (side-stream weight gradients at normal priority)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3prio
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_normal_$i.txt 2>&1 || exit $?
  DCA_STEP_STREAM_PRIORITY=high timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_high_$i.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_normal.txt 2>&1 || exit $?
DCA_STEP_STREAM_PRIORITY=high timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_high.txt 2>&1 || exit $?
for f in $O/*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
