# round 6: large-tile MFMA GEMM -- numerics, then timing against hipBLASLt, then kernel stats
set -o pipefail
OUT=gpurun_out/r6h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gemm.py > $OUT/bench.jsonl 2> $OUT/bench.err || exit 1
