#!/bin/bash
# Usage (GPU box): bash tools/ab_trace.sh <tag> "ENV=a" "ENV=b" ...
# bench.py --no-cpu under rocprofv3 --kernel-trace per environment; steady-state per-kernel table.
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abt_$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $out/run_$i.json 2> $out/run_$i.err || { echo "FAILED: $cfg"; tail -5 $out/run_$i.err; exit 1; }
  f=$(find /tmp/abt_$i -name '*kernel_trace.csv' | head -1)
  cp $f $out/trace_$i.csv
  python3 -c "import json,sys; d=json.loads(open('$out/run_$i.json').read().strip().splitlines()[-1]); print('== %-30s value=%.4g gpu_ms=%.3f frac=%.4f' % (sys.argv[1], d['value'], d['roofline']['gpu_ms_per_step'], d['roofline']['frac']))" "$cfg"
  python3 tools/ktrace.py $out/trace_$i.csv --last 10 > $out/ktrace_$i.txt
  grep -v "k_hist \|k_emit\|k_flags\|k_scan\|at::native\|rocclr\|k_init_slots\|k_conc_reset\|k_hot_reset\|k_cluster_nodes" $out/ktrace_$i.txt
done
