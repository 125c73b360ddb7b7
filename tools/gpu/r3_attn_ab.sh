# dK/dV query tile 32 vs 64: numerics, attention micro-bench, GPT-2 step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3attn
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "attention or attn" > $O/pytest.log 2>&1 || exit $?
DCA_ATTN_DKDV_QT=32 timeout -k 10 200 python tools/bench_attn.py > $O/attn_qt32.txt 2>&1 || exit $?
DCA_ATTN_FWD_KT=128 timeout -k 10 200 python tools/bench_attn.py > $O/attn_fkt128.txt 2>&1 || exit $?
DCA_ATTN_FWD_KT=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "attention or attn" > $O/pytest_fkt128.log 2>&1 || exit $?
timeout -k 10 200 python tools/bench_attn.py > $O/attn_qt64.txt 2>&1 || exit $?
DCA_ATTN_XCD_REMAP=0 timeout -k 10 200 python tools/bench_attn.py > $O/attn_noxcd.txt 2>&1 || exit $?
DCA_ATTN_DQ_KT=128 timeout -k 10 200 python tools/bench_attn.py > $O/attn_dqkt128.txt 2>&1 || exit $?
DCA_ATTN_DQ_KT=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "attention or attn" > $O/pytest_dqkt128.log 2>&1 || exit $?
DCA_ATTN_FWD_PIPE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py -k "attention or attn" > $O/pytest_pipe.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt2_qt64.txt 2>&1 || exit $?
tail -2 $O/pytest.log; grep -h "" $O/attn_qt32.txt $O/attn_qt64.txt $O/attn_fkt128.txt $O/attn_noxcd.txt $O/attn_pipe.txt | grep tflops; tail -1 $O/pytest_fkt128.log; tail -1 $O/pytest_pipe.log; grep -h -o "\"value\": [0-9.]*" $O/gpt2_qt64.txt
timeout -k 10 400 python tools/bench_asha.py --trace > $O/asha_trace.txt 2>&1 || exit $?
grep -h "startup\|metric" $O/asha_trace.txt | cut -c1-220
