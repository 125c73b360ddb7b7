# round-3 batch: full GPU test tier, attention tile A/B, space-to-depth stem (find + A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3big
( while sleep 20; do date >> gpurun_out/r3big/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3big/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r3big/pytest_gpu.log
# a test assertion (rc 1) still lets the measurements run; a fault / abort / timeout ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/r3_stem.sh || exit $?
bash tools/gpu/r3_attn_ab.sh || exit $?
