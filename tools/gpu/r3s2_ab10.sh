# env-knob A/B after LPT: dK/dV 32-query tiles, forward sub-tile-pair pipelining off
set -o pipefail
O=gpurun_out/s2ab10
mkdir -p $O
SH="32,1024,16,64;8,2048,16,64;4,4096,8,128"
for i in 1 2; do
  for v in "base" "DCA_ATTN_DKDV_QT=32" "DCA_ATTN_FWD_PIPE=0"; do
    env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/attn_${v%%=*}_$i.txt 2>&1 || exit $?
    echo "## $v $i"; grep -h '"pass"' $O/attn_${v%%=*}_$i.txt | cut -c1-130
  done
done
