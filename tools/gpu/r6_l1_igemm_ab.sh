# round 6: layer1 64->256 1x1 forward + BN on the implicit-GEMM kernel with fused statistics
# (choice forced via DCA_CONV_CHOICES) vs the shipped decision (MIOpen + BN reduce), same box
set -o pipefail
OUT=gpurun_out/r6l1
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_shipped_$i.log 2>&1 || exit 1
  DCA_CONV_CHOICES=tools/gpu/choices_l1_igemm.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_igemm_$i.log 2>&1 || exit 1
done
