#!/bin/bash
# Usage (GPU box): bash tools/r04_pmc_k.sh <tag> <kernel regex> [bench args...] -- rocprofv3 counter passes
# (one --pmc run each, kernel trace only) over the C3 bench for the kernels matching the regex; the
# per-dispatch averages are printed by tools/pmc_summary.py.
set -o pipefail
export TMPDIR=/tmp
tag=$1; rx=$2; shift 2
out=gpurun_out/pmck_$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d /tmp/pmck_${tag}_$i -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 4 --warmup 1 "$@" > $out/bench_$i.out 2>&1 || { echo "pass $i failed"; tail -5 $out/bench_$i.out; exit 1; }
  find /tmp/pmck_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
cat $out/summary.txt | head -80
