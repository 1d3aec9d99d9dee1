#!/bin/bash
# Usage (GPU box): bash tools/ab_local.sh <tag> <config> "ENV=a" "ENV=b" ... -- a local configuration's bench line
# (no CPU leg) under each environment, two runs each, interleaved; one line per run: ms per step.
set -o pipefail
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python3 bench.py --config $cfg --no-cpu > $out/ab_${i}_$rep.json 2> $out/ab_${i}_$rep.err || { echo "FAILED: $e"; tail -5 $out/ab_${i}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$out/ab_${i}_$rep.json')); print('[%s] ms %.3f gpu_ms %.3f' % (sys.argv[1], d['ms_per_step'], d['roofline']['gpu_ms_per_step']))" "$e"
  done
done
