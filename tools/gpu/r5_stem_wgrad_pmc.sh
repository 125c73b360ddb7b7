# round 5: PMC pass over the stem weight-gradient kernel (LDS conflicts / waits / MFMA busy)
set -o pipefail
OUT=gpurun_out/r5w3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/pmc -o run -- python tools/probe_stem_wgrad.py > $OUT/pmc.log 2>&1 || exit 1
