# round 6: ResNet-50 bench, same box: shipped files before the fix (broken TunableOp row) vs the
# fixed GEMM results with the re-timed chooser (layer1 64->256 1x1 forward on MIOpen) vs the fixed
# results with that forward kept on the (now correct, rocBLAS) GEMM
set -o pipefail
OUT=gpurun_out/r6fixab
mkdir -p $OUT
T=determined_clone_amd/ops/tuned
cp $T/gemm_gfx950.csv $OUT/fixed.csv
cp $T/conv_choices_gfx950.json $OUT/fixed_choices.json
for i in 1 2; do
  cp ab_old_gemm.csv $T/gemm_gfx950.csv && cp ab_old_choices.json $T/conv_choices_gfx950.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_broken_$i.log 2>&1 || exit 1
  cp $OUT/fixed.csv $T/gemm_gfx950.csv && cp $OUT/fixed_choices.json $T/conv_choices_gfx950.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_fixedlib_$i.log 2>&1 || exit 1
  cp ab_gemm_choices.json $T/conv_choices_gfx950.json
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/rn_fixedgemm_$i.log 2>&1 || exit 1
done
