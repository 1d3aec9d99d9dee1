#!/bin/bash
# Local-path A/B (GPU box): the local parity tests, then bench.py --config $CFG under each environment (2 runs each).
# Usage: CFG=c2 bash tools/r05_local_ab.sh <tag> "ENV=a" "ENV=b" ...
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05lab}; shift
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_local_parity_gpu.py tests/test_configs_fullsize_gpu.py tests/test_param_args_gpu.py tests/test_sharding.py > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $out/pytest.log | head; exit 1; }
for rep in 1 2; do
  for envs in "$@"; do
    env $envs timeout -k 10 300 python3 bench.py --config ${CFG:-c2} --no-cpu > $out/cfg.json 2> $out/cfg.err || { echo "FAIL [$envs]"; tail -5 $out/cfg.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/cfg.json').read().strip().splitlines()[-1]); p=d.get('parity_sample') or {}; print('[$envs] ms %.3f value %.3e mism %s' % (d['ms_per_step'], d['value'], p.get('mismatches')))"
  done
done
