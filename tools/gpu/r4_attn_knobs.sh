#!/bin/bash
# attention knob sweep after the branch-free prefetch change (round-3 choices re-checked):
# workgroup order, forward / dQ key tiles, dK/dV query tile, D=128 forward pipelining
set -o pipefail
O=gpurun_out/r4knobs
mkdir -p $O
SH="16,1024,16,64;8,2048,16,64;4,4096,8,128"
run() {  # label, env...
  local label=$1; shift
  echo "## $label" >> $O/bench.log
  env "$@" timeout -k 10 200 python tools/bench_attn.py --shapes "$SH" >> $O/bench.log 2>&1 || exit 1
}
for r in 1 2; do
  run "default r$r" DCA_X=0
  run "order=xcd r$r" DCA_ATTN_ORDER=xcd
  run "fwd_kt=128 r$r" DCA_ATTN_FWD_KT=128
  run "dq_kt=128 r$r" DCA_ATTN_DQ_KT=128
  run "dq_pipe r$r" DCA_ATTN_DQ_PIPE=1
  run "dkdv_qt=32 r$r" DCA_ATTN_DKDV_QT=32
  run "pipe128 r$r" DCA_ATTN_FWD_PIPE128=1
done
python3 - <<'PY'
import json, collections
rows = collections.defaultdict(lambda: collections.defaultdict(list))
label = None
for line in open("gpurun_out/r4knobs/bench.log"):
    if line.startswith("## "):
        label = line[3:].rsplit(" r", 1)[0].strip()
    elif '"pass"' in line:
        d = json.loads(line)
        rows[(d["S"], d["D"], d["pass"])][label].append(d["tflops"])
for k, v in sorted(rows.items()):
    print(k, {lab: round(sum(x) / len(x), 1) for lab, x in v.items()})
PY
