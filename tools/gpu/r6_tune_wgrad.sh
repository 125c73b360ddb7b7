# round 6: MIOpen exhaustive tuning of the ResNet-50 weight gradients (one set per call) on a private DB copy
set -o pipefail
SET=${1:-3x3}
OUT=gpurun_out/r6v_$SET
mkdir -p $OUT/db $OUT/cache
cp determined_clone_amd/ops/tuned/miopen/db/* $OUT/db/
cp determined_clone_amd/ops/tuned/miopen/cache/* $OUT/cache/
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/$OUT/db MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/$OUT/cache
timeout -k 10 300 python tools/tune_wgrad_miopen.py time $SET > $OUT/before.jsonl 2> $OUT/before.err || exit 1
MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 900 python tools/tune_wgrad_miopen.py tune $SET > $OUT/tune.jsonl 2> $OUT/tune.err || exit 1
timeout -k 10 300 python tools/tune_wgrad_miopen.py time $SET > $OUT/after.jsonl 2> $OUT/after.err || exit 1
