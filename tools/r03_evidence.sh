#!/bin/bash
# Usage (GPU box): bash tools/r03_evidence.sh <tag> -- PMC traffic passes over the C3 bench, a kernel trace of the
# same bench command with its per-kernel summary and timeline, and the side-stream priority A/B.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03ev}
out=gpurun_out/$tag
mkdir -p $out
bash tools/pmc_bench.sh $tag --no-cpu --steps 5 --warmup 1 > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -4 $out/pmc.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof_bench.err || { tail -20 $out/prof_bench.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/kstats.py $out/kernel_stats.csv > $out/kstats.txt
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
head -12 $out/ktrace.txt
bash tools/r03_ab.sh ${tag}_ab "SGA_SIDE_PRIO=0" "SGA_SIDE_PRIO=1"
