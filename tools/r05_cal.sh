#!/bin/bash
# Round-5 calibration (GPU box): record-access patterns of the cold flows phase (tools/calib/recbench),
# then the C3 bench under a kernel trace (one batch's timeline).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05cal}
mkdir -p $out
for wg in 256 512; do
  timeout -k 10 120 ./tools/calib/recbench 700000 $wg | tee -a $out/recbench.jsonl || exit 1
done
timeout -k 10 120 ./tools/calib/recbench 350000 256 | tee -a $out/recbench.jsonl || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05cal -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
f=$(find /tmp/r05cal -name '*kernel_trace.csv' | head -1)
cp $f $out/kernel_trace.csv
python3 tools/timeline.py $out/kernel_trace.csv > $out/timeline.txt
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 > $out/ktrace.txt
cat $out/timeline.txt
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
