#!/bin/bash
# Runs one gpurun call, retrying only while the pool has no free box (exit code 3); any other outcome ends it.
# Usage: bash tools/gpurun_retry.sh <timeout> '<command>'
t=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
