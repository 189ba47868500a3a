#!/bin/bash
# Retry a gpurun call only when the infrastructure reports a transient failure (box not ready /
# no slot); never retries a command that actually ran.   usage: scripts/gpurun_retry.sh TAG TIMEOUT CMD
TAG=$1; T=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_$TAG.txt 2>&1
  rc=$?
  if grep -q "status=transient\|no box or slot\|backing off" /tmp/gpurun_$TAG.txt && ! grep -q "status=ok" /tmp/gpurun_$TAG.txt; then
    sleep $((60 + 30 * i)); continue
  fi
  break
done
cat /tmp/gpurun_$TAG.txt | tail -c 3000
exit $rc
