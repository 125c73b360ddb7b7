# attention kernels at the GPT-2 in-step shape (B32 S1024 H16 D64 causal): SQ stall counters, one pass
set -o pipefail
O=gpurun_out/s2pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
  -d $GRAFT_REPO_ROOT/$O/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py --shapes "32,1024,16,64" --iters 3 > $GRAFT_REPO_ROOT/$O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC \
  -d $GRAFT_REPO_ROOT/$O/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py --shapes "32,1024,16,64" --iters 3 > $GRAFT_REPO_ROOT/$O/p2.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && for p in p1 p2; do f=$(find $O/$p -name 'run_counter_collection.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "attn" not in n: continue
    k = n.split("(")[0].replace("void dca::(anonymous namespace)::", "")
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, " ".join(f"{c}={v / max(1, cnt[(k, c)]):.4g}" for c, v in sorted(d.items())))
PY
done
