#!/bin/bash
# gpurun_retry.sh OUT TIMEOUT SCRIPT: run `bash SCRIPT` on a GPU box, retrying
# only while the pool has no box free (nothing ran, nothing charged)
out=$1; to=$2; script=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "bash $script" > $out 2>&1
  if grep -q "no free box\|slot(s) on this pod are busy\|stopped responding\|backing off\|no box" $out; then
    sleep 90
  else
    exit 0
  fi
done
