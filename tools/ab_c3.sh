#!/bin/bash
# Usage (GPU box): bash tools/ab_c3.sh <tag> "ENV=a" "ENV=b" ...  -- C3 bench A/B under kernel traces + timelines
set -o pipefail
tag=${1:-r03ab}; shift
export TMPDIR=/tmp
bash tools/ab_trace.sh $tag "$@" || exit 1
i=0
for cfg in "$@"; do
  i=$((i+1))
  python3 tools/timeline.py gpurun_out/$tag/trace_$i.csv 4 | grep -v copyBuffer > gpurun_out/$tag/timeline_$i.txt
  grep -h "fz phases" gpurun_out/$tag/run_$i.err | tail -2 || true
done
