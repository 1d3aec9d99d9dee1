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
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "${PMC_REGEX:-k_(classify|rs64_|runs_|flows|results|scan_|lim_|hs_|hot_)}" -d /tmp/pmc_${tag}_$i -o run --output-format csv -- python3 bench.py "$@" > $out/bench_$i.out 2>&1 || exit $?
  find /tmp/pmc_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
python3 tools/pmc_summary.py $out --steps-from $out/bench_1.out --json $out/traffic.json > $out/summary.txt
