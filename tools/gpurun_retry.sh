#!/bin/bash
# Host-side wrapper: run gpurun once, and again (up to 4 tries, 60 s apart)
# only when gpurun reports an infrastructure transient in which the command
# never started (no box, box lost while being prepared).  A command that ran
# and failed is never retried.  usage: tools/gpurun_retry.sh TIMEOUT 'command'
R=$(cd "$(dirname "$0")/.." && pwd)
T=$1; shift
for i in $(seq 1 ${TRIES:-4}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_retry.log 2>&1
  rc=$?
  grep -v "every call sends\|^\[gpurun\] sending" /tmp/gpurun_retry.log
  if grep -q "status=transient" /tmp/gpurun_retry.log && grep -q "run 0.0s\|run Nones" /tmp/gpurun_retry.log; then
    sleep ${WAIT:-60}
    continue
  fi
  exit $rc
done
exit $rc
