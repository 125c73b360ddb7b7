# record the CIFAR-10 search's conv shapes (widths 32/48/64, train + eval) in the shipped MIOpen
# find DB / kernel cache, copy them back, then the ASHA bench with the agent's seeded copy
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3cifar
mkdir -p $O/db
export MIOPEN_USER_DB_PATH=$PWD/determined_clone_amd/ops/tuned/miopen/db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/determined_clone_amd/ops/tuned/miopen/cache
for w in 32 48 64; do for hd in 256 512; do
  timeout -k 10 300 python tools/probe_trial_startup.py --find --width $w --hidden $hd > $O/find_w${w}_h${hd}.txt 2>&1 || exit $?
done; done
for w in 32 64; do timeout -k 10 120 python tools/probe_trial_startup.py --width $w > $O/warm_w$w.txt 2>&1 || exit $?; done
cp -a determined_clone_amd/ops/tuned/miopen/db/. $O/db/ && cp -a determined_clone_amd/ops/tuned/miopen/cache/. $O/db/
unset MIOPEN_USER_DB_PATH MIOPEN_CUSTOM_CACHE_DIR
timeout -k 10 400 python tools/bench_asha.py --trace > $O/asha.txt 2>&1 || exit $?
grep -h total_s $O/*.txt | cut -c1-250; grep -h 'startup\|"metric"' $O/asha.txt | cut -c1-200
