# A/B: attention built with / without the SLP vectorizer (DCA_OPS_SO), alternating; step-stream priority on ResNet-50 and GPT-2
set -o pipefail
O=gpurun_out/s2ab1
mkdir -p $O
SH="32,1024,16,64;16,1024,16,64;8,2048,16,64;4,4096,8,128"
for i in 1 2; do
  for v in slp noslp; do
    DCA_OPS_SO=$PWD/ab_slp/_C_$v.so timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/attn_${v}_$i.txt 2>&1 || exit $?
    echo "## $v $i"; grep -h '"pass"' $O/attn_${v}_$i.txt | cut -c1-130
  done
done
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_normal_$i.txt 2>&1 || exit $?
  DCA_STEP_STREAM_PRIORITY=high timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_high_$i.txt 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_normal.txt 2>&1 || exit $?
DCA_STEP_STREAM_PRIORITY=high timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_high.txt 2>&1 || exit $?
for f in $O/rn_*.txt $O/gpt_*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
