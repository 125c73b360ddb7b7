set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r3_probe_start.sh || exit $?
O=gpurun_out/r3attn2
mkdir -p $O
timeout -k 10 200 python tools/bench_attn.py > $O/attn_default.txt 2>&1 || exit $?
DCA_ATTN_DQ_KT=128 timeout -k 10 200 python tools/bench_attn.py > $O/attn_dqkt128.txt 2>&1 || exit $?
DCA_ATTN_DQ_KT=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "attention or attn" > $O/pytest_dqkt128.log 2>&1 || exit $?
grep -h bwd $O/attn_default.txt $O/attn_dqkt128.txt; tail -1 $O/pytest_dqkt128.log
