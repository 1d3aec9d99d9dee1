#!/bin/bash
# Usage (GPU box): bash tools/r03_full.sh <tag> -- whole GPU suite, smoke, then the C3 bench line
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03full}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $out/pytest.log | head -30; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.4f cpu %.4g' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value']))"
