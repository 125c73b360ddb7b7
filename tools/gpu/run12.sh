# MIOpen exhaustive tuning (perf-db SEARCH) of the ResNet-50 bs256 bf16 NHWC convolutions.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out/miopen_tuned
cp -r tools/miopen/db tools/miopen/cache gpurun_out/miopen_tuned/
export MIOPEN_USER_DB_PATH=$ROOT/gpurun_out/miopen_tuned/db MIOPEN_CUSTOM_CACHE_DIR=$ROOT/gpurun_out/miopen_tuned/cache
MIOPEN_FIND_ENFORCE=SEARCH MIOPEN_LOG_LEVEL=5 timeout -k 10 850 python bench.py --steps 3 --warmup 2 > gpurun_out/r12_tune.log 2>&1
echo "tune rc=$?"
tail -2 gpurun_out/r12_tune.log
timeout -k 10 250 python bench.py --steps 30 --warmup 10 2>&1 | tee gpurun_out/r12_bench_tuned.txt | tail -2
