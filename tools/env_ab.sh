#!/bin/bash
# A/B a profiling knob: bash tools/env_ab.sh <tag> VAR v1 v2 ...  (GPU box) - kernel times per value
set -o pipefail
tag=$1; var=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  export $var=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${tag}_$v -o run --output-format csv -- python3 bench.py --no-cpu > $out/bench_$v.json 2> $out/prof_$v.err || { tail -5 $out/prof_$v.err; exit 1; }
  find /tmp/prof_${tag}_$v -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace_$v.csv \;
  echo "== $var=$v"; python3 -c "import json;d=json.load(open('$out/bench_$v.json'));r=d['roofline'];print('value %.3e gpu_ms %.3f'%(d['value'],r['gpu_ms_per_step']))"
  python3 tools/ktrace.py $out/kernel_trace_$v.csv --last 10 | grep -E "k_hot|k_cold" | head -12
done
