#!/bin/bash
# Usage (on the GPU box): bash tools/quick_gpu.sh <tag>  -- GPU tests, bench (no CPU leg), kernel stats
set -o pipefail
tag=${1:-q}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -5 $out/pytest.log
[ $rc = 0 ] || { grep -E 'Error|assert|FAIL' $out/pytest.log | head -20; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu > $out/bench.json || exit 1
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value %.4g gpu_ms %.3f frac %.4f'%(d['value'],d['roofline']['gpu_ms_per_step'],d['roofline']['frac']))"
bash tools/prof_bench.sh $tag --no-cpu --steps 5 --warmup 1 || exit 1
python3 tools/kstats.py gpurun_out/prof_$tag/run_kernel_stats.csv | grep -E 'k_(classify|rs64|scan|row_scan|runs|flows|results|hs_|hot_)'
