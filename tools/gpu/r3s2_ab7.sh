# A/B builds (DCA_OPS_SO): LayerNorm backward register budget (base 169 VGPR / occ 2; lnocc 144 / occ 3;
# lnw4 128 + 68 B spill / occ 4) x DCA_LN_BWD_BLOCKS; tests first on the in-tree (lnocc) build
set -o pipefail
O=gpurun_out/s2ab7
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for v in base lnocc lnw4; do
  for b in 512 768 1024; do
    DCA_LN_BWD_BLOCKS=$b DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 200 python3 tools/bench_tx_bwd.py > $O/tx_${v}_$b.txt 2>&1 || exit $?
    echo "## tx $v blocks=$b $(grep -h 'ln_bwd' $O/tx_${v}_$b.txt | head -2 | cut -c1-120 | tr '\n' ' ')"
  done
done
for v in base lnocc; do
  DCA_OPS_SO=$PWD/ab/_C_$v.so timeout -k 10 300 python3 tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_${v}.txt 2>&1 || exit $?
  echo "gpt $v $(grep -h -o '"value": [0-9.]*' $O/gpt_${v}.txt)"
done
