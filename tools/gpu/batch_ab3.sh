# ResNet-50 bench: default (bs 1024 per GPU) vs 512 with the shipped MIOpen find/perf DB (no tuning
# expected: each run's wall time is printed)
set -o pipefail
mkdir -p gpurun_out/batch_ab3
( while sleep 30; do date +%T >> gpurun_out/batch_ab3/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 200 python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/batch_ab3/import.txt 2>&1 || exit 1
for b in 1024 512 1024 512; do
  ( time timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 8 ) > gpurun_out/batch_ab3/b$b.$RANDOM.txt 2>&1 || exit 1
done
