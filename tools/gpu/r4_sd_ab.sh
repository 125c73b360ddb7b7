#!/bin/bash
# SD-2 UNet step: which round-4 change moved it (113 img/s vs 124 at the end of round 3)?
# default vs channels_last wgrad targets off vs the old extension (attention before the
# branch-free prefetch) vs no side-stream wgrad, alternating on one box
set -o pipefail
O=gpurun_out/r4sdab
mkdir -p $O
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 tools/bench_diffusion.py --steps 10 --warmup 3 > $O/run.txt 2>&1 || { tail -20 $O/run.txt; exit 1; }
  echo "## $label: $(grep '"mode"' $O/run.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["images_per_s"], d["ms_per_step"])')"
}
for r in 1 2; do
  run "default r$r" DCA_X=0
  run "cl_targets=0 r$r" DCA_WGRAD_STREAM_CL=0
  run "old_ext r$r" DCA_OPS_SO=$PWD/ab/_C_old.so
  run "side_stream=0 r$r" DCA_WGRAD_STREAM=0
  run "igemm_wgrad=0 r$r" DCA_IGEMM_WGRAD=0
  run "keepalive=0 r$r" DCA_WGRAD_KEEPALIVE=0
done
