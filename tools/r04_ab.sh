#!/bin/bash
# Usage (GPU box): bash tools/r04_ab.sh <tag> "<env A>" "<env B>" ... -- the C3 bench line (no CPU leg, no
# host-buffer batches) under each environment, three runs each, interleaved, ms per step printed.
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for rep in 1 2 3; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 200 python3 bench.py --no-cpu --no-e2e > $out/ab_${i}_$rep.json 2> $out/ab_${i}_$rep.err || { echo "FAIL [$envs]"; tail -5 $out/ab_${i}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab_${i}_$rep.json').read().strip().splitlines()[-1]); print('[%s] ms %.4f' % ('$envs', d['ms_per_step']))"
  done
done
