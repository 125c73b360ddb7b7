# A/B builds (DCA_OPS_SO): base = HEAD attention, rowc = dK/dV row constants as initial accumulators
set -o pipefail
O=gpurun_out/s2ab4
mkdir -p $O
SH="32,1024,16,64;16,1024,16,64;8,2048,16,64;4,4096,8,128"
for i in 1 2; do
  for v in base rowc; do
    DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" --only bwd > $O/attn_${v}_$i.txt 2>&1 || exit $?
    echo "## $v $i"; grep -h '"pass"' $O/attn_${v}_$i.txt | cut -c1-130
  done
done
for v in base rowc; do
  DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_$v.txt 2>&1 || exit $?
  echo "gpt $v $(grep -h -o '"value": [0-9.]*' $O/gpt_$v.txt)"
done
