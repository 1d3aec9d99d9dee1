#!/bin/bash
# Kernel stats of one local configuration's bench (GPU box): bash tools/r05_cfgprof.sh <tag> <config>
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/$1; cfg=$2
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/cp_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 > $out/$cfg.json 2> $out/$cfg.err || { tail -5 $out/$cfg.err; exit 1; }
f=$(find /tmp/cp_$cfg -name '*kernel_stats.csv' | head -1)
cp $f $out/${cfg}_kstats.csv
python3 - $out/${cfg}_kstats.csv <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:18]:
    m = re.search(r"(k_\w+(<[^>]*>)?)\(", r["Name"])
    print(f"{(m.group(1) if m else r['Name'][:40]):40s} calls {r['Calls']:>6s} total_ms {float(r['TotalDurationNs'])/1e6:9.2f} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
python3 -c "import json; d=json.loads(open('$out/$cfg.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])"
