# ResNet-50 bench bs1024: MIOpen find per process (cudnn.benchmark) vs immediate mode from the
# shipped find DB -- throughput and process wall time
set -o pipefail
mkdir -p gpurun_out/find_ab
( while sleep 30; do date +%T >> gpurun_out/find_ab/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 200 python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/find_ab/import.txt 2>&1 || exit 1
for mode in 0 1 0; do
  ( time DCA_CONV_BENCHMARK=$mode timeout -k 10 400 python bench.py --steps 20 --warmup 8 ) > gpurun_out/find_ab/bench$mode.$RANDOM.txt 2>&1 || exit 1
done
