#!/bin/bash
# which MIOpen solvers run eagerly vs under stream capture (MIOpen info log)
set -o pipefail
mkdir -p gpurun_out
MIOPEN_LOG_LEVEL=6 timeout -k 10 240 python -u tools/probe_graph_miopen.py > gpurun_out/graph_probe_log.txt 2>&1
rc=$?
python - <<'PY'
import re
txt = open("gpurun_out/graph_probe_log.txt", errors="replace").read()
parts = re.split(r"=== PHASE (\w+)", txt)
for name, body in zip(parts[1::2], parts[2::2]):
    lines = [l for l in body.splitlines() if re.search(r"olver|Algorithm|algo|Find|workspace|Workspace|Immediate|Fallback", l)]
    print("#####", name, len(lines))
    for l in lines[:60]:
        print(l[:300])
PY
exit $rc
