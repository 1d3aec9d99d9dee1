#!/bin/bash
# Usage (on the GPU box): bash tools/pmc_bench.sh <tag> [bench args...]
# 1) FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/calib/pmccal, 2 GiB tables);
# 2) one rocprofv3 --pmc pass per counter group over the headline bench (kernel-trace only, no other
#    trace domains); 3) a kernel trace of the same bench for durations; 4) the per-kernel table.
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out/cal
timeout -k 10 60 ./tools/calib/pmccal > $out/cal/cal.out 2>&1 || exit $?
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-include-regex "k_cal_" -d /tmp/pmccal_${tag}_$i -o run --output-format csv -- ./tools/calib/pmccal > /dev/null 2>&1 || exit $?
  find /tmp/pmccal_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/cal/counters_$i.csv \;
done
python3 tools/pmc_cal.py $out/cal --json $out/cal/cal.json || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "${PMC_REGEX:-k_}" -d /tmp/pmc_${tag}_$i -o run --output-format csv -- python3 bench.py "$@" > $out/bench_$i.out 2>&1 || exit $?
  find /tmp/pmc_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/pmct_${tag} -o run --output-format csv -- python3 bench.py "$@" > $out/bench_trace.out 2>&1 || exit $?
find /tmp/pmct_${tag} -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/pmc_summary.py $out --steps-from $out/bench_1.out --cal $out/cal/cal.json --trace $out/kernel_trace.csv \
  --json $out/traffic.json > $out/summary.txt
tail -30 $out/summary.txt
