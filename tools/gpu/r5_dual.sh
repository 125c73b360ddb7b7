# round 5: dual-BN (bn3 + projection-shortcut BN) fusion: numerics, same-box A/B, step breakdown
set -o pipefail
ROOT=$(pwd)
OUT=gpurun_out/r5d
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "dual or bn_act_forward" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/dual_$i.log 2>&1 || exit 1
  DCA_BN_DUAL=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/sep_$i.log 2>&1 || exit 1
  DCA_CONV_CHOICES=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/timed_$i.log 2>&1 || exit 1
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 8 --warmup 4 > $ROOT/$OUT/prof_bench.log 2>&1 && \
cd $ROOT && f=$(find $OUT/prof -name 'run_kernel_trace.csv' | head -1) && \
python3 tools/analyze_trace.py $f 4 2 sgd_kernel "" bn_ > $OUT/breakdown.txt && rm -f $f
