# round 5: HIP-graph runner without forced deterministic MIOpen solvers: graph tests, CIFAR trial
# probe, then the ASHA full search with graphed trials vs eager
set -o pipefail
OUT=gpurun_out/r5v
mkdir -p $OUT
( while sleep 30; do date +%T >> $OUT/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 150 python tools/probe_cifar_graph.py 300 1 > $OUT/probe_graph.json 2> $OUT/probe_graph.err || exit 1
timeout -k 10 150 python tools/probe_cifar_graph.py 300 0 > $OUT/probe_eager.json 2> $OUT/probe_eager.err || exit 1
timeout -k 10 400 python tools/bench_asha.py --gpus 1 --hip-graph 1 > $OUT/asha_graph.json 2> $OUT/asha_graph.err || exit 1
timeout -k 10 400 python tools/bench_asha.py --gpus 1 --hip-graph 0 > $OUT/asha_eager.json 2> $OUT/asha_eager.err || exit 1
