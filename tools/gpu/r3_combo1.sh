set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3conv
timeout -k 10 300 python tools/bench_conv3x3.py > gpurun_out/r3conv/conv3x3.txt 2>&1 || exit $?
bash tools/gpu/r3_var2.sh || exit $?
bash tools/gpu/r3_tx.sh
