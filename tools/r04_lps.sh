#!/bin/bash
# Usage (GPU box): bash tools/r04_lps.sh <tag> -- k_llru_ps: the CacheMap GPU tests, then C4 full mode with the
# chunked replay (default) and with k_llru (SGA_LRU_PS=0).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04lps}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_param_lru_gpu.py tests/test_pseg_gpu.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python3 bench.py --config c4full --steps 2 --warmup 1 --no-cpu > $out/c4full_ps.json 2> $out/c4full_ps.err || { tail -5 $out/c4full_ps.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/c4full_ps.json')); print('c4full ps', d['value'], 'ms %.1f' % d['ms_per_step'])"
