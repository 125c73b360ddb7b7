# round 6: MIOpen exhaustive tuning of the stem convolution (forward + weight gradient) on a private DB copy
set -o pipefail
OUT=gpurun_out/r6u
mkdir -p $OUT/db $OUT/cache
cp determined_clone_amd/ops/tuned/miopen/db/* $OUT/db/
cp determined_clone_amd/ops/tuned/miopen/cache/* $OUT/cache/
export MIOPEN_USER_DB_PATH=$GRAFT_REPO_ROOT/$OUT/db MIOPEN_CUSTOM_CACHE_DIR=$GRAFT_REPO_ROOT/$OUT/cache
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 200 python tools/tune_stem_miopen.py time > $OUT/before.json 2> $OUT/before.err || exit 1
MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 700 python tools/tune_stem_miopen.py tune > $OUT/tune.json 2> $OUT/tune.err || exit 1
timeout -k 10 200 python tools/tune_stem_miopen.py time > $OUT/after.json 2> $OUT/after.err || exit 1
