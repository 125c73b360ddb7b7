# ResNet-50 bench: images per GPU 768 / 1024 vs 512 (layer4 GEMMs fill 256 CUs only at large M;
# first run of a new size runs MIOpen find for its 3x3/7x7 shapes; the updated user find/perf DB is
# copied back so the tuned solvers ship in-tree)
set -o pipefail
mkdir -p gpurun_out/batch_ab2
( while sleep 30; do date +%T >> gpurun_out/batch_ab2/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
for b in 1024 768; do
  ( time timeout -k 10 800 python bench.py --batch $b --steps 10 --warmup 12 ) > gpurun_out/batch_ab2/b$b.first.txt 2>&1 || exit 1
  mkdir -p gpurun_out/batch_ab2/miopen && cp -r tools/miopen/db tools/miopen/cache gpurun_out/batch_ab2/miopen/
done
for b in 512 1024 768 512 1024; do
  timeout -k 10 400 python bench.py --batch $b --steps 20 --warmup 8 > gpurun_out/batch_ab2/b$b.$RANDOM.txt 2>&1 || exit 1
done
