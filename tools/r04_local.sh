#!/bin/bash
# Usage (GPU box): bash tools/r04_local.sh <tag> [configs] -- the local-path GPU suite, then the device-resident
# config lines (bench.py --config <cfg> --no-cpu) with their ms per step.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04l}; shift
cfgs=${@:-c1 c2 c4 c5b}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 700 python3 -u -m pytest tests/test_local_parity_gpu.py tests/test_pseg_gpu.py tests/test_param_args_gpu.py \
    tests/test_param_lru_gpu.py tests/test_configs_fullsize_gpu.py tests/test_local_device_gpu.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for c in $cfgs; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu > $out/config_$c.json 2> $out/config_$c.err || { tail -5 $out/config_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/config_$c.json')); print('$c', d['value'], 'ms %.3f' % d['ms_per_step'])"
done
