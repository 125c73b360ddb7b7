# ResNet-50 bs1024: conv chooser decisions (DCA_CONV_DEBUG=1)
set -o pipefail
O=gpurun_out/s2chooser
mkdir -p $O
DCA_CONV_DEBUG=1 timeout -k 10 240 python3 bench.py --steps 3 --warmup 2 > $O/bench.txt 2> $O/chooser.txt || exit $?
grep "conv chooser" $O/chooser.txt | sort | uniq | head -60
