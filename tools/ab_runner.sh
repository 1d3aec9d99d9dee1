#!/bin/bash
# Usage (GPU box): bash tools/ab_runner.sh <tag> <pytest files...> -- "ENV=a" "ENV=b" ...
# The listed GPU tests, then the C3 bench line under each environment (2 runs each, interleaved), then a kernel
# trace (one batch's timeline) of the first environment.
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
tests=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do tests+=("$1"); shift; done
shift
if [ ${#tests[@]} -gt 0 ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread "${tests[@]}" > $out/pytest.log 2>&1
  rc=$?
  tail -3 $out/pytest.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $out/pytest.log | head -20; grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/pytest.log && exit 1; fi
fi
for rep in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    extra="--no-parity"; [ $rep = 1 ] && extra=""
    env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e $extra > $out/ab_${i}_$rep.json 2> $out/ab_${i}_$rep.err || { echo "FAIL [$envs]"; tail -5 $out/ab_${i}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab_${i}_$rep.json').read().strip().splitlines()[-1]); p=d.get('parity_sample') or {}; print('[$envs] ms %.4f gpu_ms %.4f mism %s' % (d['ms_per_step'], d['roofline']['gpu_ms_per_step'], p.get('mismatches')))"
  done
done
env $1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/abtr -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-parity --steps 10 --warmup 3 > $out/tr.json 2> $out/tr.err || { tail -5 $out/tr.err; exit 1; }
f=$(find /tmp/abtr -name '*kernel_trace.csv' | head -1)
cp $f $out/trace.csv
python3 tools/timeline.py $out/trace.csv > $out/timeline.txt
cat $out/timeline.txt
