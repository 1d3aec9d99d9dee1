#!/bin/bash
# Usage (on the GPU box): bash tools/pmc_bench.sh <tag> [bench args...]
# One rocprofv3 --pmc pass per counter group (kernel-trace only, no other trace
# domains), restricted to the engine's kernels; keeps the per-dispatch counter CSVs.
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-include-regex 'k_(classify|rs_scatter|rs_hist|runs_up|runs_down|flows|results)' -d /tmp/pmc_${tag}_$i -o run --output-format csv -- python3 bench.py "$@" > $out/bench_$i.out 2>&1 || exit $?
  find /tmp/pmc_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
