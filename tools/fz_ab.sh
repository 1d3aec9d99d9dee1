#!/bin/bash
# A/B of hot-path kernel phases (profiling only: results are wrong when a phase is skipped).
# Usage (GPU box): bash tools/fz_ab.sh "<SGA_FZ_DEBUG values>" "<kernel regex>"
set -o pipefail
export TMPDIR=/tmp
vals=${1:-"0 1 2"}; rx=${2:-k_cold_fused}
mkdir -p gpurun_out/fz
for d in $vals; do
  SGA_FZ_DEBUG=$d timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/fz_$d -o run --output-format csv -- python3 bench.py --no-cpu --steps 6 --warmup 3 > gpurun_out/fz/b$d.json 2> gpurun_out/fz/b$d.err || exit 1
  f=$(find /tmp/fz_$d -name "*kernel_trace.csv" | head -1)
  echo "SGA_FZ_DEBUG=$d:"; python3 tools/ktrace.py $f --last 6 | grep -E "$rx"
done
