#!/bin/bash
# Usage (on the GPU box): bash tools/round_evidence.sh <tag>
# Everything a round's judged numbers come from, in one call: GPU tests, smoke, PMC traffic passes,
# the bench (with the CPU baseline) and a rocprofv3 kernel-trace summary of the same bench command.
set -o pipefail
tag=${1:-r}
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p $out
nproc > $out/nproc.txt; lscpu > $out/lscpu.txt 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; cat $out/smoke.log; exit 1; }
cat $out/smoke.log
bash tools/pmc_bench.sh $tag --no-cpu --steps 5 --warmup 1 || { echo "pmc failed"; exit 1; }
mkdir -p profiles && cp gpurun_out/pmc_$tag/traffic.json profiles/traffic_c3.json
tail -1 gpurun_out/pmc_$tag/summary.txt
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof_bench.err || { echo "prof failed"; tail -20 $out/prof_bench.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/kstats.py $out/kernel_stats.csv > $out/kstats.txt
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
head -24 $out/ktrace.txt
bash tools/local_configs.sh ${tag}_lc
