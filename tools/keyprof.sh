#!/bin/bash
# Key-kernel cost split (GPU box): the kernel's average duration with and without its rank pass
# (SGA_FZ_DEBUG=4 skips it; decisions are then wrong, timing only).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05kp}
mkdir -p $out
for dbg in 0 4; do
  SGA_FZ_DEBUG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kp_$dbg -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-parity --steps 4 --warmup 2 > $out/kp_$dbg.out 2>&1 || { tail -5 $out/kp_$dbg.out; exit 1; }
  f=$(find /tmp/kp_$dbg -name '*kernel_stats.csv' | head -1)
  cp $f $out/kstats_$dbg.csv
  echo "dbg=$dbg"; grep -E "k_hot_key_dense<0|k_cold_fused|k_hot_final_g|k_part_scatter" $out/kstats_$dbg.csv | cut -d, -f1-5 | cut -c1-160
done
