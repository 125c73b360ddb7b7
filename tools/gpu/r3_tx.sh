# transformer backward kernels: numerics, micro-benchmarks (LN bwd block sweep), GPT-2 end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tx
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_gpt2.py > $O/pytest.log 2>&1 || exit $?
for b in 512 1024 2048 4096; do
  DCA_LN_BWD_BLOCKS=$b timeout -k 10 120 python tools/bench_tx_bwd.py > $O/micro_$b.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt2.txt 2>&1 || exit $?
tail -3 $O/pytest.log; cat $O/micro_2048.txt; grep -h ln_bwd $O/micro_*.txt; tail -2 $O/gpt2.txt
timeout -k 10 200 python tools/bench_attn.py > $O/attn.txt 2>&1 || exit $?
cat $O/attn.txt | tail -8
