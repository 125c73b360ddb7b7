#!/bin/bash
# BN apply passes on the flat grid: rows in flight per lane (U) / block cap sweep (DCA_BN_APPLY="U,max_blocks")
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4bnsweep
mkdir -p $O
for v in default 2,1073741824 4,1073741824 8,1073741824 4,4096 8,2048; do
  if [ $v = default ]; then unset DCA_BN_APPLY; else export DCA_BN_APPLY=$v; fi
  tag=$(echo $v | tr ',' '_')
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$tag -o run -- python3 $ROOT/tools/bench_bn_kernels.py --run > $O/run_$tag.log 2>&1 || exit 1
  cd $ROOT && f=$(find $O/t_$tag -name 'run_kernel_trace.csv' | head -1) && python3 tools/bench_bn_kernels.py --trace $f > $O/sum_$tag.txt && rm -f $f || exit 1
  echo "## $v: $(tail -1 $O/sum_$tag.txt)"
done
