#!/bin/bash
# usage: tools/gpu_retry.sh <outfile> <timeout> <command...>; retries only infrastructure-transient outcomes
out=$1; shift; to=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" $out; then
    echo "attempt $i transient" >> $out.attempts; sleep 60; continue
  fi
  break
done
