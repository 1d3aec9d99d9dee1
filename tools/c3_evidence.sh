#!/bin/bash
# Usage (GPU box): bash tools/c3_evidence.sh <tag> -- the C3 bench line (CPU baseline included), then a rocprofv3
# kernel-trace summary of the same command without the CPU leg, its kernel table and one batch's timeline.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-c3e}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
tail -1 $out/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu \
    > $out/prof_bench.json 2> $out/prof_bench.err || { echo "prof failed"; tail -20 $out/prof_bench.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/kstats.py $out/kernel_stats.csv > $out/kstats.txt
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
python3 tools/timeline.py $out/kernel_trace.csv 2 > $out/timeline.txt
rm -f $out/kernel_trace.csv
head -12 $out/ktrace.txt
