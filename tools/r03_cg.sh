#!/bin/bash
# Usage (GPU box): bash tools/r03_cg.sh <tag> "<pytest files>" "ENV=a" "ENV=b" ...
#   the named GPU parity tests, then C3 bench A/B under kernel traces
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
files=$1; shift
mkdir -p gpurun_out/$tag
if [ -n "$files" ]; then
  timeout -k 10 600 python3 -u -m pytest $files -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
  rc=$?
  tail -3 gpurun_out/$tag/pytest.log
  [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$tag/pytest.log | head -30; exit 1; }
fi
if [ $# -gt 0 ]; then bash tools/r03_ab.sh ${tag}_ab "$@"; fi
