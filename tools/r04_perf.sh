#!/bin/bash
# Usage (GPU box): bash tools/r04_perf.sh <tag> [env assignments...] -- C3 perf only: k_cold_fused phase times
# (SGA_FZ_DEBUG=16), the bench line (no CPU leg, no host-buffer batches) and a kernel trace of it
# (per-kernel table + one batch's timeline).  Extra arguments are exported first (A/B knobs).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04p}; shift
for kv in "$@"; do export "$kv"; done
out=gpurun_out/$tag
mkdir -p $out
SGA_FZ_DEBUG=16 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 4 --warmup 1 > $out/fz.json 2> $out/fz.err || { tail -20 $out/fz.err; exit 1; }
grep "fz phases" $out/fz.err | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e > $out/prof_bench.json 2> $out/prof_bench.err || { tail -20 $out/prof_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/prof_bench.json').read().strip().splitlines()[-1]); print('traced: value %.4g ms %.4f' % (d['value'], d['ms_per_step']))"
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
python3 tools/timeline.py $out/kernel_trace.csv > $out/timeline.txt 2>&1 || true
cat $out/timeline.txt
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))"
