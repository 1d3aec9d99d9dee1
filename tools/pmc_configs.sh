#!/bin/bash
# Usage (GPU box): bash tools/pmc_configs.sh <tag> [configs...] -- HBM traffic per step from rocprofv3 PMC passes
# (FETCH_SIZE and WRITE_SIZE in passes of their own, kernel trace only, as MI355X_MICROARCH.md prescribes):
# calibration (tools/calib/pmccal), then per configuration two counter passes and a kernel trace of the bench
# line, summarised by tools/pmc_summary.py into gpurun_out/<tag>/traffic_<cfg>.json.
# c3: bench.py --steps 5 --warmup 1 --no-cpu --no-e2e; c2/c4/c5b: bench.py --config <cfg> --steps 2 --warmup 1 --no-cpu.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04p}; shift
cfgs=${@:-c3 c2 c4 c5b}
out=gpurun_out/$tag
mkdir -p $out/cal
timeout -k 10 60 ./tools/calib/pmccal > $out/cal/cal.out 2>&1 || { echo "calibration failed"; exit 1; }
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-include-regex "k_cal_" -d /tmp/pmccal_${tag}_$i -o run \
      --output-format csv -- ./tools/calib/pmccal > /dev/null 2>&1 || { echo "cal pass $i failed"; exit 1; }
  find /tmp/pmccal_${tag}_$i -name "*counter_collection.csv" -exec cp {} $out/cal/counters_$i.csv \;
done
python3 tools/pmc_cal.py $out/cal --json $out/cal/cal.json || exit 1
for cfg in $cfgs; do
  d=$out/$cfg
  mkdir -p $d
  if [ "$cfg" = "c3" ]; then args="--steps 5 --warmup 1 --no-cpu --no-e2e"; extra="";
  else args="--config $cfg --steps 2 --warmup 1 --no-cpu"; extra="--all-random"; fi
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex "k_" -d /tmp/pmc_${tag}_${cfg}_$i -o run \
        --output-format csv -- python3 bench.py $args > $d/bench_$i.out 2>&1 || { echo "$cfg pass $i failed"; tail -3 $d/bench_$i.out; exit 1; }
    find /tmp/pmc_${tag}_${cfg}_$i -name "*counter_collection.csv" -exec cp {} $d/counters_$i.csv \;
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pmct_${tag}_${cfg} -o run --output-format csv -- \
      python3 bench.py $args > $d/bench_trace.out 2>&1 || { echo "$cfg trace failed"; exit 1; }
  find /tmp/pmct_${tag}_${cfg} -name "*kernel_trace.csv" -exec cp {} $d/kernel_trace.csv \;
  find /tmp/pmct_${tag}_${cfg} -name "*kernel_stats.csv" -exec cp {} $d/kernel_stats.csv \;
  python3 tools/pmc_summary.py $d --steps-from $d/bench_1.out --cal $out/cal/cal.json --trace $d/kernel_trace.csv \
      $extra --json $out/traffic_$cfg.json > $d/summary.txt || { echo "$cfg summary failed"; exit 1; }
  echo "== $cfg"; tail -4 $d/summary.txt
done
