# round 6: MIOpen backward-data solver A/B (the atomic split-K asm solver zero-fills dx on the main stream)
set -o pipefail
OUT=gpurun_out/r6q
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/base_$i.log 2>&1 || exit 1
  MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/nobwdgtc_$i.log 2>&1 || exit 1
done
