#!/bin/bash
# A/B of k_cold_fused phases (profiling only): steady-state kernel time with phases skipped.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fz
for d in 0 1 2 3; do
  SGA_FZ_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/fz_$d -o run --output-format csv -- python3 bench.py --no-cpu --steps 6 --warmup 3 > gpurun_out/fz/b$d.json 2> gpurun_out/fz/b$d.err || exit 1
  f=$(find /tmp/fz_$d -name "*kernel_trace.csv" | head -1)
  echo "SGA_FZ_DEBUG=$d: $(python3 tools/ktrace.py $f --last 6 | grep k_cold_fused)"
done
