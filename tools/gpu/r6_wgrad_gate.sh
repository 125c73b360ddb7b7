# round 6: GPT-2 step with the main stream's bandwidth-bound backward kernels gated on the preceding
# side-stream weight gradient (DCA_WGRAD_GATE, ops/transformer.py) vs ungated
set -o pipefail
OUT=gpurun_out/r6gate
mkdir -p $OUT
DCA_WGRAD_GATE=gelu,ln,attn timeout -k 10 120 python -u -m pytest tests/test_transformer_ops_gpu.py tests/test_gpt2.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/pytest_gate.log 2>&1 || exit 1
for i in 1 2; do
  for g in none gelu gelu,ln gelu,ln,attn; do
    tag=$(echo $g | tr , _)
    if [ $g = none ]; then
      timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_${tag}_$i.log 2>&1 || exit 1
    else
      DCA_WGRAD_GATE=$g timeout -k 10 300 python tools/bench_gpt2.py --steps 10 --warmup 3 > $OUT/gpt2_${tag}_$i.log 2>&1 || exit 1
    fi
  done
done
