#!/bin/bash
# usage: tools/gpu_retry.sh <outfile> <timeout> <command...>
# Retries only infrastructure-transient outcomes (box not prepared / no free box / backing off),
# honouring gpurun's "retry in Ns" hint; a command that ran (any exit status) is never retried.
out=$1; shift; to=$1; shift
for i in $(seq 1 30); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" $out; then
    wait_s=$(grep -o "retry in [0-9]*s" $out | tail -1 | grep -o "[0-9]*")
    echo "attempt $i transient (wait ${wait_s:-60})" >> $out.attempts
    sleep $(( ${wait_s:-60} + 15 ))
    continue
  fi
  break
done
