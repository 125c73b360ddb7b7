set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/igemm3
mkdir -p $O
timeout -k 10 120 python tools/bench_igemm.py --check-only > $O/check.txt 2>&1 || { cat $O/check.txt; exit 1; }
for st in 2 3; do for bm in 128 256; do
  DCA_IGEMM_STAGES=$st DCA_IGEMM_BM=$bm timeout -k 10 300 python tools/bench_igemm.py > $O/bench_s${st}_bm${bm}.txt 2>&1 || { tail $O/bench_s${st}_bm${bm}.txt; exit 1; }
  echo "stages=$st bm=$bm"; grep -o '"H": [0-9]*, "cin": [0-9]*\|"ig_fwd_us": [0-9.]*\|"ig_dgrad_us": [0-9.]*\|per_step.*' $O/bench_s${st}_bm${bm}.txt | tr '\n' ' '; echo
done; done
