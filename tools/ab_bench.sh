#!/bin/bash
# Usage (on the GPU box): bash tools/ab_bench.sh "ENV1=a ENV2=b" "ENV1=c" ...
# bench.py --no-cpu once per environment setting (under rocprofv3 kernel stats); value, GPU ms/step
# and the engine kernels' average durations.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/ab_$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/ab/run_$i.json 2> gpurun_out/ab/run_$i.err || { echo "FAILED: $cfg"; tail -5 gpurun_out/ab/run_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/run_$i.json').read().strip().splitlines()[-1]); print('%-40s value=%.4g gpu_ms=%.3f frac=%.4f' % (sys.argv[1], d['value'], d['roofline']['gpu_ms_per_step'], d['roofline']['frac']))" "$cfg"
  python3 tools/kstats.py $(find /tmp/ab_$i -name '*kernel_stats.csv') | grep -E 'k_(classify|rs64|scan|row_scan|runs|flows|results)'
done
