#!/bin/bash
# Usage (on the GPU box): bash tools/ab_bench.sh "ENV1=a ENV2=b" "ENV1=c" ...
# Runs bench.py --no-cpu once per environment setting; prints value and GPU ms/step.
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python3 bench.py --no-cpu > gpurun_out/ab/run_$i.json 2> gpurun_out/ab/run_$i.err || { echo "FAILED: $cfg"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/run_$i.json').read().strip().splitlines()[-1]); print('%-40s value=%.4g gpu_ms=%.3f frac=%.4f' % (sys.argv[1], d['value'], d['roofline']['gpu_ms_per_step'], d['roofline']['frac']))" "$cfg"
done
