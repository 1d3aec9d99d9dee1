#!/bin/bash
# Usage (GPU box): bash tools/local_cfg.sh <tag> <config...>  -- bench.py --config lines (one JSON each)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-lc}; shift
out=gpurun_out/$tag
mkdir -p $out
for c in "$@"; do
  timeout -k 10 400 python3 bench.py --config $c > $out/$c.json 2> $out/$c.err || { echo "bench $c failed"; tail -20 $out/$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/$c.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};cb=d.get('cpu_baseline') or {};print('$c', '%.3e'%d['value'], d['unit'], 'ms/step %.2f'%d['ms_per_step'], 'frac', r.get('frac'), 'cpu', cb.get('value'), 'cpu1', cb.get('value_1thread'), 'cpuT', cb.get('value_threads'))"
done
