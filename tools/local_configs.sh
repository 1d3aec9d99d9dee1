#!/bin/bash
# Usage (GPU box): bash tools/local_configs.sh <tag>
# bench.py --config c1 c2 c4 c5a c5b (device-resident local entries), one JSON line each.
set -o pipefail
tag=${1:-lc}
out=gpurun_out/$tag
mkdir -p $out
for c in ${CONFIGS:-c1 c2 c4 c5a c5b c4full}; do
  timeout -k 10 240 python3 bench.py --config $c > $out/$c.json 2> $out/$c.err || { echo "bench $c failed"; tail -20 $out/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/$c.json'));r=d.get('roofline') or {};cb=d.get('cpu_baseline') or {};print('$c', '%.3e'%d['value'], d['unit'], 'frac', r.get('frac'), 'cpu', cb.get('value'))"
done
