# attention causal workgroup order A/B: XCD remap (default) vs heaviest-first (DCA_ATTN_ORDER=lpt)
set -o pipefail
O=gpurun_out/s2lpt${1:-}
mkdir -p $O
SH="16,1024,16,64;32,1024,16,64;8,2048,16,64;4,4096,8,128"
DCA_ATTN_ORDER=lpt timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for mode in xcd lpt xcd lpt; do
  DCA_ATTN_ORDER=$mode timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/$mode.txt 2>&1 || exit $?
  echo "## $mode"; grep -h '"pass"' $O/$mode.txt | cut -c1-120
done
