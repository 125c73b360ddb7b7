#!/bin/bash
# bench.py under allocator / stream settings, optionally with HBM held by another process.
# usage: bash tools/gpu/r4_bench_mem.sh "label|ENV=V ...|hogGB" ...
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --gpus 1 --steps 10 --warmup 3"
OUT=gpurun_out/benchmem.txt; ERR=gpurun_out/benchmem.err
: > $OUT; : > $ERR
for case in "$@"; do
  IFS='|' read -r label envs gb <<< "$case"
  HOG=""
  if [ "$gb" != "0" ]; then
    rm -f gpurun_out/hog_ready
    python -c "
import torch, time
x = torch.empty(int($gb * 2**30), dtype=torch.uint8, device='cuda'); x.fill_(1); torch.cuda.synchronize()
open('gpurun_out/hog_ready', 'w').write('ok'); time.sleep(400)" &
    HOG=$!
    for i in $(seq 1 120); do [ -f gpurun_out/hog_ready ] && break; sleep 1; done
  fi
  echo "## $label (env: $envs, other process holds $gb GB)" | tee -a $ERR >> $OUT
  env $envs DCA_BENCH_MEM_WAIT_S=0 timeout -k 10 300 $B >> $OUT 2>> $ERR
  rc=$?
  if [ -n "$HOG" ]; then kill $HOG; wait $HOG 2>/dev/null; fi
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; break; }
done
python - <<'PY'
import json
for l in open("gpurun_out/benchmem.txt"):
    if l.startswith("##"): print(l.strip()); continue
    try: d = json.loads(l)
    except Exception: continue
    print("  value", d["value"], "ms", d["ms_per_step"], d.get("diagnostics"))
PY
grep -E "^##|step_ms" $ERR | cut -c1-220
