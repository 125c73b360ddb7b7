# round 6: MIOpen weight-gradient solver A/B -- the atomic split-K asm solver (zero-fill + fp32 cast
# around every call) vs the solvers MIOpen picks without it
set -o pipefail
OUT=gpurun_out/r6g
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/base_$i.log 2>&1 || exit 1
  MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/nogtc_$i.log 2>&1 || exit 1
done
MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC=1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/det_1.log 2>&1 || exit 1
