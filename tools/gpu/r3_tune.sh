# TunableOp tuning runs for the GPT-2 and ResNet-50 benchmark GEMMs, then replay A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3tune
mkdir -p $O
PYTORCH_TUNABLEOP_VERBOSE=1 DCA_GEMM_TUNE=$O/gpt2.csv timeout -k 10 600 python tools/bench_gpt2.py --steps 2 --warmup 1 > $O/tune_gpt2.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_VERBOSE=1 DCA_GEMM_TUNE=$O/resnet.csv timeout -k 10 600 python bench.py --steps 2 --warmup 1 > $O/tune_resnet.log 2>&1 || exit $?
wc -l $O/*.csv
