# round 6: PMC of the 3x3 implicit GEMM with the side stream idle (conv weights frozen) -- the isolated
# counterpart of r6_contention.sh's in-step passes
set -o pipefail
OUT=gpurun_out/r6s
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES"
P2="FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES"
for m in freeze_conv normal; do
  timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex "conv_fwd_kernel" --output-format csv -d $OUT/pmc1_$m -o run -- python tools/probe_contention.py --mode $m --steps 2 --warmup 2 > $OUT/pmc1_$m.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc $P2 --kernel-include-regex "conv_fwd_kernel" --output-format csv -d $OUT/pmc2_$m -o run -- python tools/probe_contention.py --mode $m --steps 2 --warmup 2 > $OUT/pmc2_$m.log 2>&1 || exit 1
done
