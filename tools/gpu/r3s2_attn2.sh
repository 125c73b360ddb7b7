# attention after -fno-slp-vectorize: tests + throughput (GPT-2 in-step shape B32 first)
set -o pipefail
O=gpurun_out/s2attn2${1:-}
mkdir -p $O
SH="32,1024,16,64;16,1024,16,64;8,2048,16,64;4,4096,8,128"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/attn.txt 2>&1 || exit $?
grep -h '"pass"' $O/attn.txt | cut -c1-130
