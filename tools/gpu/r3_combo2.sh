# TunableOp tuning runs for the GPT-2 and ResNet-50 benchmark GEMMs, then replay A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tune
mkdir -p $O
PYTORCH_TUNABLEOP_VERBOSE=1 DCA_GEMM_TUNE=$O/gpt2.csv timeout -k 10 600 python tools/bench_gpt2.py --steps 2 --warmup 1 > $O/tune_gpt2.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_VERBOSE=1 DCA_GEMM_TUNE=$O/resnet.csv timeout -k 10 600 python bench.py --steps 2 --warmup 1 > $O/tune_resnet.log 2>&1 || exit $?
wc -l $O/*.csv
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
#timeout -k 10 400 python tools/bench_conv3x3.py --find --only-stem > gpurun_out/r3smi/stem_find.txt 2>&1 || exit $?
cat gpurun_out/r3smi/stem_find.txt
