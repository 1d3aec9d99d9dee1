#!/bin/bash
# Usage (GPU box): bash tools/kprof_configs.sh <tag> [configs...] -- rocprofv3 kernel-trace summary of each local
# configuration's bench line (no CPU baseline), kernel_stats.csv + a short-name table per configuration.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-kp}; shift
out=gpurun_out/$tag
mkdir -p $out
for cfg in ${@:-c2 c4 c5b}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kp_${tag}_$cfg -o run --output-format csv -- \
      python3 bench.py --config $cfg --steps ${KP_STEPS:-5} --warmup 1 --no-cpu > $out/$cfg.json 2> $out/$cfg.err \
      || { echo "$cfg failed"; tail -5 $out/$cfg.err; exit 1; }
  find /tmp/kp_${tag}_$cfg -name "*kernel_stats.csv" -exec cp {} $out/${cfg}_kernel_stats.csv \;
  python3 tools/kstats.py $out/${cfg}_kernel_stats.csv > $out/${cfg}_kstats.txt
  echo "== $cfg $(python3 -c "import json;print(round(json.load(open('$out/$cfg.json'))['ms_per_step'],3))") ms/step"
  head -14 $out/${cfg}_kstats.txt
done
