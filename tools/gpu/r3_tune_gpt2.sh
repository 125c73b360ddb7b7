# TunableOp tuning of the GPT-2-medium benchmark GEMMs, then a replay A/B (default heuristic vs tuned)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tune
mkdir -p $O
( while sleep 20; do date >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
[ -f $O/gpt2.csv ] || cp tools/tuned_seed/gpt2.csv $O/gpt2.csv 2>/dev/null || true
DCA_GEMM_TUNE=$O/gpt2.csv timeout -k 10 900 python tools/bench_gpt2.py --steps 2 --warmup 1 > $O/tune_gpt2.log 2>&1 || exit $?
mkdir -p determined_clone_amd/ops/tuned && cp $O/gpt2.csv determined_clone_amd/ops/tuned/gemm_gfx950.csv
DCA_GEMM_TUNED=0 timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt2_default.txt 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt2_tuned.txt 2>&1 || exit $?
md5sum determined_clone_amd/ops/tuned/gemm_gfx950.csv $O/gpt2.csv > $O/md5_after_replay.txt
grep -h metric $O/gpt2_default.txt $O/gpt2_tuned.txt | cut -c1-200
