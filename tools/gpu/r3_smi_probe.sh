# Does a concurrent SMI sampler (like a driver's gpu-busy probe) slow the ResNet bench?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3smi
mkdir -p $O
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/plain_1.log 2>&1 || exit $?
( for i in $(seq 1 40); do rocm-smi --showuse --showmemuse --json > /dev/null 2>&1; sleep 1; done ) &
SAMPLER=$!
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocmsmi_2.log 2>&1; rc=$?
kill $SAMPLER 2>/dev/null; wait $SAMPLER 2>/dev/null
[ $rc -eq 0 ] || exit $rc
( for i in $(seq 1 40); do amd-smi metric --usage --json > /dev/null 2>&1; sleep 1; done ) &
SAMPLER=$!
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/amdsmi_3.log 2>&1; rc=$?
kill $SAMPLER 2>/dev/null; wait $SAMPLER 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/plain_4.log 2>&1 || exit $?
grep -h -o '"value": [0-9.]*' $O/*.log
