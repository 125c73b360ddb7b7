# per-kernel times of the transformer backward microbench (LN bwd vs its dgamma/dbeta column reduce)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/s2proftx
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bench_tx_bwd.py > $O/tx.txt 2>&1 || { tail -20 $O/tx.txt; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
head -12 "$f" | cut -c1-220
