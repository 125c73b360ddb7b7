# round 6: SD UNet step, several processes on one box, each traced, to see whether the slow mode is
# per process and which kernels differ
set -o pipefail
OUT=gpurun_out/r6sdm
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$i -o run -- python tools/bench_diffusion.py --steps 10 --warmup 3 > $OUT/run$i.log 2>&1 || exit 1
  rm -f $OUT/p$i/run_kernel_trace.csv
done
