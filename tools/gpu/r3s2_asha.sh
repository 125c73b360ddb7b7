# ASHA trials/hr with this session's code (start-up trace)
set -o pipefail
O=gpurun_out/s2asha
mkdir -p $O
timeout -k 10 400 python tools/bench_asha.py --trace > $O/asha.txt 2>&1 || exit $?
grep -h '"metric"' $O/asha.txt | cut -c1-300; grep -h startup $O/asha.txt
