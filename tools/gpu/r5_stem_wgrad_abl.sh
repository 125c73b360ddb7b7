# round 5: stem weight-gradient timing-only ablations (1: no row loads after the first, 2: no MFMA/LDS reads)
set -o pipefail
OUT=gpurun_out/r5w6
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for a in 0 1 2 3; do
  DCA_STEM_WGRAD_ABL=$a timeout -k 10 120 python tools/bench_stem_s2d.py > $OUT/micro$a.txt 2>&1 || exit 1
  echo "abl=$a $(grep 'hip stem_wgrad' $OUT/micro$a.txt)" >> $OUT/abl.txt
done
