#!/bin/bash
# Usage (GPU box): bash tools/r03_gpu.sh <tag> [pytest -k expr]  -- GPU tests, then the C3 bench under a kernel trace
set -o pipefail
tag=${1:-r03}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$2" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > $out/pytest.log 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
fi
rc=$?
tail -4 $out/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL|error" $out/pytest.log | head -30; exit 1; }
bash tools/ab_trace.sh ${tag}_t "SGA_X=0" || exit 1
python3 tools/timeline.py $out/../${tag}_t/trace_1.csv 4 | grep -v copyBuffer > $out/timeline.txt
head -30 $out/timeline.txt
