# dsat engine hook on the GPU + the transformer / conv GPU tests after this session's kernel edits
set -o pipefail
O=gpurun_out/s2dsat
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dsat_asha.py -m gpu > $O/pytest_dsat.txt 2>&1 || { tail -40 $O/pytest_dsat.txt; exit 1; }
grep -E "passed|failed" $O/pytest_dsat.txt | tail -1
