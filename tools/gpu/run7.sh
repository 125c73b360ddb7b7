set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/probe_gpt2.py gpt2-small 4 2 2>&1 | tee gpurun_out/r7_small.txt
timeout -k 10 300 python tools/probe_gpt2.py gpt2-medium 8 2 2>&1 | tee gpurun_out/r7_medium.txt
