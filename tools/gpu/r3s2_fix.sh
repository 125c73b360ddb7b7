# residual layout check fix: graph tests (cudnn-disabled ResNet, chooser timing) + conv tests + BN tests
set -o pipefail
O=gpurun_out/s2fix
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_gpu.py tests/test_conv_gpu.py tests/test_ops_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
