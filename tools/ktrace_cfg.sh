#!/bin/bash
# Usage (GPU box): bash tools/ktrace_cfg.sh <tag> <config> [env...] -- kernel trace of a local config bench
set -o pipefail
export TMPDIR=/tmp
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 > $out/$cfg.json 2> $out/$cfg.err || { tail -20 $out/$cfg.err; exit 1; }
f=$(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -1)
cp $f $out/${cfg}_kernel_stats.csv
python3 - "$out/${cfg}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-60s calls=%6s total_ms=%10.2f avg_us=%10.1f" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
