#!/bin/bash
# Kernel stats of one bench config: bash tools/cfg_prof.sh <tag> <config> [steps]  (GPU box)
set -o pipefail
tag=$1; c=$2; k=${3:-2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --config $c --steps $k --warmup 1 --no-cpu > $out/$c.json 2> $out/$c.err || { tail -5 $out/$c.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/${c}_kernel_stats.csv \;
python3 -c "import json;d=json.load(open('$out/$c.json'));r=d['roofline'];print('$c', '%.3e'%d['value'], 'ms/step %.2f gpu_ms %.2f'%(d['ms_per_step'], r['gpu_ms_per_step']))"
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$out/${c}_kernel_stats.csv")))
rows.sort(key=lambda r:-float(r["TotalDurationNs"]))
for r in rows[:14]: print("%-40s calls=%5s total_ms=%9.2f avg_us=%9.1f"%(r["Name"][:40], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e3))
PY
