# round 6: fused MLP projection + dGELU backward in isolation, with kernel stats
set -o pipefail
OUT=gpurun_out/r6f
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/bench_mlp_dgelu.py > $OUT/mlp.jsonl 2> $OUT/mlp.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python tools/bench_mlp_dgelu.py --iters 5 > $OUT/prof.log 2>&1 || exit 1
