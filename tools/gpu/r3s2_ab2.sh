# A/B: step-stream priority on ResNet-50 and GPT-2 (with this session's attention), alternating
set -o pipefail
O=gpurun_out/s2ab2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_normal_$i.txt 2>&1 || exit $?
  DCA_STEP_STREAM_PRIORITY=high timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_high_$i.txt 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_normal_$i.txt 2>&1 || exit $?
  DCA_STEP_STREAM_PRIORITY=high timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_high_$i.txt 2>&1 || exit $?
done
for f in $O/rn_*.txt $O/gpt_*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
