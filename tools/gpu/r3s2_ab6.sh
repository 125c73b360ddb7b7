# A/B builds (DCA_OPS_SO): base vs lnpf (LayerNorm backward with next-row prefetch); tests first
set -o pipefail
O=gpurun_out/s2ab6
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_ops_gpu.py tests/test_groupnorm_gpu.py tests/test_conv_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in base lnpf; do
  DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 200 python3 tools/bench_tx_bwd.py > $O/tx_$v.txt 2>&1 || exit $?
  echo "## tx $v"; grep -h 'ln_bwd' $O/tx_$v.txt | head -4 | cut -c1-150
done
for i in 1 2; do
  for v in base lnpf; do
    DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_${v}_$i.txt 2>&1 || exit $?
    echo "gpt $v $i $(grep -h -o '"value": [0-9.]*' $O/gpt_${v}_$i.txt)"
  done
done
