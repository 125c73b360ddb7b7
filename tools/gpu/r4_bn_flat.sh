#!/bin/bash
# BN apply passes: channel-group-fastest flat grid (default) vs the 2-D grid (DCA_BN_APPLY_FLAT=0):
# numerics, per-kernel bandwidth at every ResNet-50 BN shape, and the ResNet-50 step, same box
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4bnflat
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_conv_gpu.py tests/test_transformer_ops_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  cd /tmp && DCA_BN_APPLY_FLAT=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$v -o run -- python3 $ROOT/tools/bench_bn_kernels.py --run > $O/run$v.log 2>&1 || exit 1
  cd $ROOT && f=$(find $O/t$v -name 'run_kernel_trace.csv' | head -1) && python3 tools/bench_bn_kernels.py --trace $f > $O/summary$v.txt && rm -f $f || exit 1
  echo "## FLAT=$v"; grep -E '"C": (1024|2048|512)|per_step' $O/summary$v.txt
done
for r in 1 2; do
  for v in 1 0; do
    DCA_BN_APPLY_FLAT=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > $O/bench$v.log 2>&1 || exit 1
    echo "## bench FLAT=$v round $r: $(tail -1 $O/bench$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
# attention backward per-kernel times at the GPT-2 shape (what else runs inside the timed bwd)
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/attn -o run --output-format csv -- python3 $ROOT/tools/bench_attn.py --gpt2 --only bwd > $O/attn_run.log 2>&1 || exit 1
cd $ROOT && f=$(find $O/attn -name 'run_kernel_stats.csv' | head -1) && cut -d, -f1-8 $f | head -14
# grouped-query attention throughput (Llama-style 32 query / 8 K/V heads at D 128) vs MHA
cd $ROOT && timeout -k 10 200 python3 tools/bench_attn.py --shapes "2,4096,32,128" > $O/gqa.log 2>&1 && \
timeout -k 10 200 python3 tools/bench_attn.py --shapes "2,4096,32,128" --kv-heads 8 >> $O/gqa.log 2>&1 || exit 1
grep '"pass"' $O/gqa.log
