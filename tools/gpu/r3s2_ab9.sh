# env-knob A/B after the LPT order / LN prefetch: attention key tiles (fwd / dQ 128) and LN-bwd block count, in the GPT-2 step
set -o pipefail
O=gpurun_out/s2ab9
mkdir -p $O
SH="32,1024,16,64;8,2048,16,64"
for v in "base" "DCA_ATTN_FWD_KT=128" "DCA_ATTN_DQ_KT=128"; do
  env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/attn_${v%%=*}.txt 2>&1 || exit $?
  echo "## $v"; grep -h '"pass"' $O/attn_${v%%=*}.txt | cut -c1-130
done
for i in 1 2; do
  for v in "base" "DCA_LN_BWD_BLOCKS=2048" "DCA_LN_BWD_BLOCKS=512"; do
    env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_${v##*=}_$i.txt 2>&1 || exit $?
    echo "gpt $v $i $(grep -h -o '"value": [0-9.]*' $O/gpt_${v##*=}_$i.txt)"
  done
done
