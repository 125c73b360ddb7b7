# TunableOp tuning of the ResNet-50 benchmark's library GEMMs (pointwise convs as GEMMs, classifier),
# then a replay A/B (default heuristic vs tuned results merged with the GPT-2 ones)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tune
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat_rn.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
DCA_GEMM_TUNE=$O/resnet.csv timeout -k 10 1000 python bench.py --steps 2 --warmup 1 > $O/tune_resnet.log 2>&1 || exit $?
python tools/tune_gemms.py $O/resnet.csv > $O/merge.txt 2>&1 || exit $?
cp determined_clone_amd/ops/tuned/gemm_gfx950.csv $O/merged.csv
DCA_GEMM_TUNED=0 timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_default.txt 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_tuned.txt 2>&1 || exit $?
grep -h '"metric"' $O/rn_default.txt $O/rn_tuned.txt | cut -c1-150
timeout -k 10 400 python tools/bench_conv3x3.py --find --only-stem > $O/stem_find.txt 2>&1 || exit $?
cat $O/stem_find.txt
