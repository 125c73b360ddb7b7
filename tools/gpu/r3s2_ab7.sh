# ResNet-50 bs1024: conv weight gradients on the side stream (default) vs inline (DCA_WGRAD_STREAM=0), alternating
set -o pipefail
O=gpurun_out/s2ab7
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_side_$i.txt 2>&1 || exit $?
  DCA_WGRAD_STREAM=0 timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_inline_$i.txt 2>&1 || exit $?
done
for f in $O/rn_*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
