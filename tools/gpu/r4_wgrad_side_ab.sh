#!/bin/bash
# 3x3 / stem weight gradients on the side stream (channels_last direct targets): tests + same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_conv_gpu.py tests/test_graph_gpu.py tests/test_ops_gpu.py > gpurun_out/wgside_tests.log 2>&1
rc=$?; tail -2 gpurun_out/wgside_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/wgside_ab.txt
for r in 1 2; do for v in new old; do
  echo "## $v round $r" >> gpurun_out/wgside_ab.txt
  if [ $v = old ]; then E="DCA_WGRAD_STREAM_CL=0"; else E="DCA_X=1"; fi
  env $E timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/wgside_ab.txt 2>/dev/null || exit 1
done; done
python - <<'PY'
import json
for l in open("gpurun_out/wgside_ab.txt"):
    if l.startswith("##"): print(l.strip()); continue
    try: d = json.loads(l)
    except Exception: continue
    print("  ", d["value"], "img/s", d["ms_per_step"], "ms", d.get("diagnostics"))
PY
