# attention kernels: available counters + one PMC pass (SQ block only) on the GPT-2 shape
set -o pipefail
mkdir -p gpurun_out/attn_pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/attn_pmc/avail.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
  -d gpurun_out/attn_pmc/p1 -o run --output-format csv -- python3 tools/bench_attn.py --gpt2 --iters 5 > gpurun_out/attn_pmc/p1.log 2>&1
echo "p1 exit $?"
