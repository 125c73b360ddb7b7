# round 6: kernel traces of the ResNet-50 bench with the pre-fix tuned files (wrong layer1 GEMM) and
# the fixed ones, same box, to attribute the step-time difference
set -o pipefail
OUT=gpurun_out/r6fixprof
mkdir -p $OUT
T=determined_clone_amd/ops/tuned
cp $T/gemm_gfx950.csv $OUT/fixed.csv
cp $T/conv_choices_gfx950.json $OUT/fixed_choices.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
cp ab_old_gemm.csv $T/gemm_gfx950.csv && cp ab_old_choices.json $T/conv_choices_gfx950.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/broken -o run -- python bench.py --steps 5 --warmup 3 > $OUT/broken.log 2>&1 || exit 1
cp $OUT/fixed.csv $T/gemm_gfx950.csv && cp $OUT/fixed_choices.json $T/conv_choices_gfx950.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/fixed -o run -- python bench.py --steps 5 --warmup 3 > $OUT/fixed.log 2>&1 || exit 1
