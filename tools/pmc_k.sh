#!/bin/bash
# PMC passes over chosen kernels of the headline bench, one rocprofv3 run per counter set.
# Usage (GPU box): bash tools/pmc_k.sh <tag> <kernel regex> "<set1>" ["<set2>" ...]
set -o pipefail
tag=$1; rx=$2; shift 2
export TMPDIR=/tmp
out=gpurun_out/pmck_$tag
mkdir -p $out
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d /tmp/pmck_${tag}_$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 2 > $out/bench_$i.out 2>&1 || exit $?
  find /tmp/pmck_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/counters_$i.csv \;
done
python3 tools/pmc_summary.py $out > $out/summary.txt
cat $out/summary.txt
