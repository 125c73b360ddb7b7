# TunableOp tuning of the SD-2-shaped UNet train-step GEMMs, merged into the shipped file, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tune_sd
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
DCA_GEMM_TUNE=$O/sd.csv timeout -k 10 900 python tools/bench_diffusion.py --steps 2 --warmup 1 > $O/tune_sd.log 2>&1 || exit $?
python tools/tune_gemms.py $O/sd.csv > $O/merge.txt 2>&1 || exit $?
cp determined_clone_amd/ops/tuned/gemm_gfx950.csv $O/merged.csv
DCA_GEMM_TUNED=0 timeout -k 10 300 python tools/bench_diffusion.py > $O/sd_default.txt 2>&1 || exit $?
timeout -k 10 300 python tools/bench_diffusion.py > $O/sd_tuned.txt 2>&1 || exit $?
grep -h images_per_s $O/sd_default.txt $O/sd_tuned.txt | cut -c1-200
