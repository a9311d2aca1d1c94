#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool answers "no box / slot free" or a transient
# infrastructure failure before the command ran (nothing charged).  A call whose command ran is never repeated.
#   bash tools/gpurun_wait.sh <log> <timeout_s> '<command>'
log=${1:?log}
lim=${2:?timeout}
cmd=${3:?command}
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && grep -q "run 0.0s\|run Nones\|infrastructure event" "$log"; then
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
