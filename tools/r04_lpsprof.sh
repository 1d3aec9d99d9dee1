#!/bin/bash
# Usage (GPU box): bash tools/r04_lpsprof.sh <tag> -- C4 full mode: the kernel split (rocprofv3) and the k_llru_ps
# phase split (SGA_LRU_PROF=1, wave 0's phases).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04lpsprof}
mkdir -p $out
[ -z "$NOPROF" ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c4full -- python3 bench.py --config c4full --steps 2 \
    --warmup 1 --no-cpu > $out/c4full.json 2> $out/c4full.err || { tail -5 $out/c4full.err; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print("%-28s calls %6s total %10.2f ms avg %9.1f us %5.1f%%" % (r["Name"][:28], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
          float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
}
SGA_LRU_PROF=1 timeout -k 10 300 python3 bench.py --config c4full --steps 2 --warmup 1 --no-cpu > $out/c4full_p.json \
    2> $out/c4full_p.err || { tail -5 $out/c4full_p.err; exit 1; }
grep lps_prof $out/c4full_p.err | tail -2
python3 -c "import json; d=json.load(open('$out/c4full_p.json')); print('c4full', d['value'])"
