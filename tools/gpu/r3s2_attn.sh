# attention: GPU numerics tests + kernel throughput (default shapes + non-causal S1024)
set -o pipefail
O=gpurun_out/s2attn${1:-}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python3 tools/bench_attn.py > $O/attn.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_attn.py --shapes "16,1024,16,64" --noncausal >> $O/attn.txt 2>&1 || exit $?
grep -h '"pass"' $O/attn.txt
