set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
mkdir -p gpurun_out/tunableop
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$ROOT/gpurun_out/tunableop/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200
timeout -k 10 600 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 8 2>&1 | tee gpurun_out/r11_gpt2_tune_m8.txt
timeout -k 10 600 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 16 2>&1 | tee gpurun_out/r11_gpt2_tune_m16.txt
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 8 2>&1 | tee gpurun_out/r11_gpt2_tuned_m8.txt
timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 4 --micro 16 2>&1 | tee gpurun_out/r11_gpt2_tuned_m16.txt
ls -la gpurun_out/tunableop
