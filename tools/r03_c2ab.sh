#!/bin/bash
# Usage (GPU box): bash tools/r03_c2ab.sh <tag> -- local parity tests, then C2 under both RateLimiter window modes
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r03c2}
out=gpurun_out/$tag
mkdir -p $out
SGA_PACE_SCAN=1 timeout -k 10 600 python3 -u -m pytest tests/test_local_parity_gpu.py tests/test_configs_fullsize_gpu.py tests/test_local_device_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc = 0 ] || { grep -E "Error|assert|FAIL" $out/pytest.log | head -20; exit 1; }
for m in 1 0; do
  SGA_PACE_SCAN=$m timeout -k 10 300 python3 bench.py --config c2 --no-cpu --steps 3 --warmup 1 > $out/c2_$m.json 2> $out/c2_$m.err || { tail -5 $out/c2_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/c2_$m.json'));print('SGA_PACE_SCAN=$m', d['ms_per_step'], '%.3g' % d['value'])"
done
