#!/bin/bash
# Round-5 evidence (GPU box), after the GPU suite: PMC traffic passes of the C3 bench, the bench line (with the
# CPU baseline), a kernel trace + stats of the same command, the batch timeline, and the local configuration lines.
set -o pipefail
tag=${1:-r05e}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
bash tools/pmc_bench.sh $tag --no-cpu --no-e2e --steps 5 --warmup 1 || { echo "pmc failed"; exit 1; }
cp gpurun_out/pmc_$tag/traffic.json profiles/traffic_c3.json
cp gpurun_out/pmc_$tag/summary.txt $out/pmc_summary.txt
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
tail -c 1500 $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof_bench.err || { echo "prof failed"; tail -20 $out/prof_bench.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/kstats.py $out/kernel_stats.csv > $out/kstats.txt
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
python3 tools/timeline.py $out/kernel_trace.csv > $out/timeline.txt
cat $out/timeline.txt
