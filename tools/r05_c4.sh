#!/bin/bash
# C4 pinned A/B (GPU box): the CacheMap tests, then bench.py --config c4 with the working tree and a variant library.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05c4}; shift
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_param_lru_gpu.py tests/test_cluster_param_gpu.py "tests/test_configs_fullsize_gpu.py::test_c4_10k_param_rules_pinned" tests/test_pseg_gpu.py > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $out/pytest.log | head; exit 1; }
for rep in 1 2; do
  for envs in "$@"; do
    env $envs timeout -k 10 300 python3 bench.py --config ${CFG:-c4} --no-cpu > $out/c4.json 2> $out/c4.err || { echo "FAIL [$envs]"; tail -5 $out/c4.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/c4.json').read().strip().splitlines()[-1]); p=d.get('parity_sample') or {}; print('[$envs] ms %.3f value %.3e mism %s' % (d['ms_per_step'], d['value'], p.get('mismatches')))"
  done
done
