# ResNet-50: conv1 dgrad accumulated into the shortcut gradient (DCA_PW_ACC_RESIDUAL=1, new default) vs separate; GPU test first
set -o pipefail
O=gpurun_out/s2ab8
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_acc_$i.txt 2>&1 || exit $?
  DCA_PW_ACC_RESIDUAL=0 timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 > $O/rn_sep_$i.txt 2>&1 || exit $?
done
for f in $O/rn_*.txt; do echo "$(basename $f) $(grep -h -o '"value": [0-9.]*' $f)"; done
