# trial start-up probe: first-batch costs in fresh processes (MIOpen caches cold / warm / shipped)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3probe
mkdir -p $O
timeout -k 10 120 python tools/probe_trial_startup.py > $O/p1_cold.txt 2>&1 || exit $?
timeout -k 10 120 python tools/probe_trial_startup.py > $O/p2_warm.txt 2>&1 || exit $?
MIOPEN_USER_DB_PATH=$PWD/determined_clone_amd/ops/tuned/miopen/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/determined_clone_amd/ops/tuned/miopen/cache timeout -k 10 120 python tools/probe_trial_startup.py > $O/p3_shipped.txt 2>&1 || exit $?
DCA_GEMM_TUNED=0 timeout -k 10 120 python tools/probe_trial_startup.py > $O/p4_untuned.txt 2>&1 || exit $?
ls -la ~/.cache/miopen 2>&1 | head -5 > $O/home_cache.txt
grep -h total_s $O/p*.txt
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_transformer_ops_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; tail -2 $O/pytest.log
