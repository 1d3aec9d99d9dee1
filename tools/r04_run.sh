#!/bin/bash
# Usage (GPU box): bash tools/r04_run.sh <tag> [pytest selection...]
# GPU tests (the selection, default the whole -m gpu suite), smoke, the C3 bench line, then a kernel
# trace of the same bench without the host-buffer batches (--no-e2e: every dispatch set is a timed or
# warmup step) summarised by tools/ktrace.py and tools/timeline.py.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04}; shift
sel=${@:-tests}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $out/pytest.log | head -30; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.4f cpu %.4g e2e %.4g' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['end_to_end_host_buffers']['value']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e > $out/prof_bench.json 2> $out/prof_bench.err || { tail -20 $out/prof_bench.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
head -14 $out/ktrace.txt
python3 tools/timeline.py $out/kernel_trace.csv > $out/timeline.txt 2>&1 || true
