# attention forward/backward throughput sweep: S at fixed tokens, causal and not; batch scaling at S1024
set -o pipefail
O=gpurun_out/s2sweep${1:-}
mkdir -p $O
SH="32,512,16,64;16,1024,16,64;8,2048,16,64;4,4096,16,64;64,1024,16,64;4,1024,16,64"
timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" > $O/causal.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_attn.py --shapes "$SH" --noncausal > $O/noncausal.txt 2>&1 || exit $?
grep -h '"pass"' $O/causal.txt $O/noncausal.txt
