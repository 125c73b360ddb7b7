#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_graph_gpu.py > gpurun_out/graph_tests.txt 2>&1 &&
timeout -k 10 300 python -u tools/probe_graph_gpu.py --resnet > gpurun_out/graph_probe_10step.txt 2>&1
rc=$?
tail -8 gpurun_out/graph_tests.txt; cat gpurun_out/graph_probe_10step.txt | head -20
exit $rc
