# round 5: record the chooser decisions inside the real bench process, add bs256 + UNet, A/B
set -o pipefail
OUT=gpurun_out/r5e
mkdir -p $OUT
rm -f $OUT/choices.json
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
DCA_CONV_CHOICES=0 DCA_CONV_DUMP=$OUT/choices.json timeout -k 10 200 python bench.py --steps 5 --warmup 3 > $OUT/record.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/dump_conv_choices.py --out $OUT/choices.json --batches 256 > $OUT/dump.log 2>&1 || exit 1
for i in 1 2; do
  DCA_CONV_CHOICES=$OUT/choices.json timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/shipped_$i.log 2>&1 || exit 1
  DCA_CONV_CHOICES=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/timed_$i.log 2>&1 || exit 1
done
