#!/bin/bash
# One kernel family, SQ counters only (issue vs wait).  Usage: bash tools/pmc_one.sh <tag> <regex>
set -o pipefail
tag=$1; rx=$2
export TMPDIR=/tmp
out=gpurun_out/pmc1_$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d /tmp/pmc1_${tag}_$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 2 > $out/bench_$i.out 2>&1 || exit $?
  find /tmp/pmc1_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
python3 tools/pmc_summary.py $out > $out/summary.txt
cat $out/summary.txt
