# dK/dV row-constant accumulators (new default) + dQ pipelined pair A/B (DCA_ATTN_DQ_PIPE), tests both ways
set -o pipefail
O=gpurun_out/s2ab3
mkdir -p $O
SH="32,1024,16,64;16,1024,16,64;8,2048,16,64;4,4096,8,128"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
DCA_ATTN_DQ_PIPE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k flash > $O/pytest_pipe.txt 2>&1 || { tail -30 $O/pytest_pipe.txt; exit 1; }
tail -1 $O/pytest.txt $O/pytest_pipe.txt
for i in 1 2; do
  for v in 0 1; do
    DCA_ATTN_DQ_PIPE=$v timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" --only bwd > $O/attn_${v}_$i.txt 2>&1 || exit $?
    echo "## dq_pipe=$v $i"; grep -h '"pass"' $O/attn_${v}_$i.txt | cut -c1-130
  done
done
