#!/bin/bash
# Usage (GPU box): bash tools/r03_base.sh <tag> -- C3 bench line (with CPU baseline) + kernel trace + timeline
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03base}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json
bash tools/ab_trace.sh ${tag}_t "SGA_X=0" || exit 1
python3 tools/timeline.py gpurun_out/${tag}_t/trace_1.csv 4 | grep -v copyBuffer > $out/timeline.txt
cat $out/timeline.txt
