# round 6: ResNet-50 side-stream contention + 3x3 implicit-GEMM in-step vs main-alone PMC
set -o pipefail
OUT=gpurun_out/r6a
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_contention.py --mode normal > $OUT/normal.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_contention.py --mode freeze_conv > $OUT/freeze.log 2>&1 || exit 1
DCA_WGRAD_STREAM=0 timeout -k 10 300 python tools/probe_contention.py --mode normal > $OUT/serial.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_normal -o run -- python tools/probe_contention.py --mode normal --steps 4 --warmup 3 > $OUT/prof_normal.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_freeze -o run -- python tools/probe_contention.py --mode freeze_conv --steps 4 --warmup 3 > $OUT/prof_freeze.log 2>&1 || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES"
P2="FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES"
for m in normal; do
  timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex "conv_fwd_kernel" --output-format csv -d $OUT/pmc1_$m -o run -- python tools/probe_contention.py --mode $m --steps 2 --warmup 2 > $OUT/pmc1_$m.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc $P2 --kernel-include-regex "conv_fwd_kernel" --output-format csv -d $OUT/pmc2_$m -o run -- python tools/probe_contention.py --mode $m --steps 2 --warmup 2 > $OUT/pmc2_$m.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
