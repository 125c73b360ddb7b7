# A/B builds (DCA_OPS_SO): base vs trpad (forward V tile padded for conflict-free transposed reads); tests + attention + GPT-2
set -o pipefail
O=gpurun_out/s2ab11
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
SH="32,1024,16,64;8,2048,16,64;4,4096,8,128;8,4096,5,64"
for i in 1 2; do
  for v in base trpad; do
    DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" --only fwd > $O/attn_${v}_$i.txt 2>&1 || exit $?
    DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 200 python3 tools/bench_attn.py --shapes "8,4096,5,64" --only fwd --noncausal >> $O/attn_${v}_$i.txt 2>&1 || exit $?
    echo "## $v $i"; grep -h '"pass"' $O/attn_${v}_$i.txt | cut -c1-140
  done
done
