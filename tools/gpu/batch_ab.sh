# ResNet-50 bench: images per GPU 256 vs 384 vs 512 (MIOpen finds new shapes during warmup; the
# updated user find/perf DB is copied back so the tuned solvers ship in-tree)
set -o pipefail
mkdir -p gpurun_out/batch_ab
( while sleep 30; do date +%T >> gpurun_out/batch_ab/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
for b in 512 384; do
  ( time timeout -k 10 700 python bench.py --batch $b --steps 20 --warmup 12 ) > gpurun_out/batch_ab/b$b.first.txt 2>&1 || exit 1
  mkdir -p gpurun_out/batch_ab/miopen && cp -r tools/miopen/db tools/miopen/cache gpurun_out/batch_ab/miopen/
done
for b in 256 512 384 256 512; do
  timeout -k 10 400 python bench.py --batch $b --steps 30 --warmup 8 > gpurun_out/batch_ab/b$b.$RANDOM.txt 2>&1 || exit 1
done
