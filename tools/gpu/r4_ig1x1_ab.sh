#!/bin/bash
# ResNet-50 bs1024: 1x1 forwards with fused BN statistics (DCA_IG1X1=auto, default) vs library (0), same box, alternating
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ig1x1_ab.txt
DCA_CONV_DEBUG=1 timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/ig1x1_choices.json 2> gpurun_out/ig1x1_choices.err || exit 1
grep "fwd1x1+bn" gpurun_out/ig1x1_choices.err | cut -c1-160
for r in 1 2; do for v in auto 0; do
  echo "## DCA_IG1X1=$v round $r" >> gpurun_out/ig1x1_ab.txt
  DCA_IG1X1=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/ig1x1_ab.txt 2>/dev/null || exit 1
done; done
python - <<'PY'
import json
for l in open("gpurun_out/ig1x1_ab.txt"):
    if l.startswith("##"): print(l.strip()); continue
    try: d = json.loads(l)
    except Exception: continue
    print("  ", d["value"], "img/s", d["ms_per_step"], "ms", d.get("diagnostics"))
PY
