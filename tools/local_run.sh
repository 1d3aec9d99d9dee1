#!/bin/bash
# Round 6 (GPU box): local-path GPU tests + config lines.  Usage: bash tools/r06_local.sh <tag> "<pytest args>" <configs...>
set -o pipefail
export TMPDIR=/tmp
tag=$1; tests=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
if [ -n "$tests" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread $tests > $out/pytest.log 2>&1
  rc=$?; tail -3 $out/pytest.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $out/pytest.log | head -20; exit 1; fi
fi
for c in "$@"; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu > $out/config_$c.json 2> $out/config_$c.err || { echo "FAIL $c"; tail -5 $out/config_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/config_$c.json').read().strip().splitlines()[-1]); print('$c', 'ms %.3f' % d['ms_per_step'], 'value %.3g' % d['value'], 'parity', d.get('parity_sample'))"
done
