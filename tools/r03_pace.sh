#!/bin/bash
# Usage (GPU box): bash tools/r03_pace.sh <tag> -- full GPU suite, the local parity tests again under
# SGA_PACE_SCAN=1, C2 lines with speculation and with the pace scan, smoke, C3 bench line
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03pace}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $out/pytest.log | head -30; exit 1; }
SGA_PACE_SCAN=1 timeout -k 10 600 python3 -u -m pytest tests/test_local_parity_gpu.py tests/test_configs_fullsize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_pace.log 2>&1
rc=$?; tail -3 $out/pytest_pace.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $out/pytest_pace.log | head -30; exit 1; }
for v in 0 1; do
  SGA_PACE_SCAN=$v timeout -k 10 400 python3 bench.py --config c2 > $out/c2_pace$v.json 2> $out/c2_pace$v.err || { tail -20 $out/c2_pace$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/c2_pace$v.json').read().strip().splitlines()[-1]);print('c2 pace$v', '%.4e'%d['value'], d['unit'], 'ms/step %.3f'%d['ms_per_step'])"
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.4f cpu %.4g' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value']))"
