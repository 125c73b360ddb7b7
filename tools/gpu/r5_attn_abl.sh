# round 5: timing-only ablations of the attention forward (DCA_ATTN_ABL bits; wrong outputs, timing
# only) + the 64-rows-per-wave variant with separated score chains
set -o pipefail
OUT=gpurun_out/r5k
mkdir -p $OUT
for i in 1 2; do
  for a in 0 1 2 4 8 15; do
    DCA_ATTN_ABL=$a timeout -k 10 120 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" > $OUT/abl_${a}_$i.jsonl 2>>$OUT/err.txt || exit 1
  done
  DCA_ATTN_FWD_W64=1 timeout -k 10 120 python tools/bench_attn.py --only fwd --shapes "16,1024,16,64;8,2048,16,64;4,4096,8,128" > $OUT/w64_$i.jsonl 2>>$OUT/err.txt || exit 1
done
