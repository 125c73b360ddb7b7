# round 5: attention forward ablations, part 2: K/V tile loads (16), + LDS stores/barriers (48), all (63)
set -o pipefail
OUT=gpurun_out/r5l
mkdir -p $OUT
for i in 1 2; do
  for a in 0 16 48 63 15; do
    DCA_ATTN_ABL=$a timeout -k 10 120 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" > $OUT/abl_${a}_$i.jsonl 2>>$OUT/err.txt || exit 1
  done
done
