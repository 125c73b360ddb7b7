#!/bin/bash
# Reproduce the 7k "slow mode": bench.py while another process still holds part of the HBM
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --gpus 1 --steps 10 --warmup 3"
hog() {  # $1 = GB to hold
  rm -f gpurun_out/hog_ready
  python -c "
import torch, time, sys
x = torch.empty(int($1 * 2**30), dtype=torch.uint8, device='cuda'); x.fill_(1); torch.cuda.synchronize()
open('gpurun_out/hog_ready', 'w').write('ok'); time.sleep(400)" &
  HOG=$!
  for i in $(seq 1 120); do [ -f gpurun_out/hog_ready ] && break; sleep 1; done
}
echo "## clean" > gpurun_out/slowmode.txt
timeout -k 10 240 $B >> gpurun_out/slowmode.txt 2>> gpurun_out/slowmode.err || exit 1
for GB in 150 180 200; do
  hog $GB
  echo "## another process holds $GB GB" >> gpurun_out/slowmode.txt
  DCA_BENCH_MEM_WAIT_S=0 timeout -k 10 300 $B >> gpurun_out/slowmode.txt 2>> gpurun_out/slowmode.err
  rc=$?
  kill $HOG; wait $HOG 2>/dev/null
  [ $rc -eq 0 ] || { echo "bench rc=$rc" >> gpurun_out/slowmode.txt; break; }
done
cat gpurun_out/slowmode.txt | cut -c1-400
grep -E "step_ms|gpu_state_mid" gpurun_out/slowmode.err | cut -c1-300
