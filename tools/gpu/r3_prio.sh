# A/B: training step on a high-priority stream (side-stream weight gradients at normal priority)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3prio
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_normal_$i.txt 2>&1 || exit $?
  DCA_STEP_STREAM_PRIORITY=high timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/rn_high_$i.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_normal.txt 2>&1 || exit $?
DCA_STEP_STREAM_PRIORITY=high timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 > $O/gpt_high.txt 2>&1 || exit $?
for f in $O/*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
# SD UNet: current defaults vs round-2 behaviour of the changed transformer paths, same box
timeout -k 10 300 python tools/bench_diffusion.py > $O/sd_now.txt 2>&1 || exit $?
DCA_ATTN_XCD_REMAP=0 DCA_ATTN_FWD_PIPE=0 DCA_ATTN_DKDV_QT=32 timeout -k 10 300 python tools/bench_diffusion.py > $O/sd_attn_r2.txt 2>&1 || exit $?
DCA_WGRAD_SPLITK=0 timeout -k 10 300 python tools/bench_diffusion.py > $O/sd_nosplitk.txt 2>&1 || exit $?
grep -h images_per_s $O/sd_*.txt
