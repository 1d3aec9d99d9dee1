#!/bin/bash
# Usage (on the GPU box): bash tools/hot_pmc.sh <tag> -- bench + kernel stats + PMC passes (no tests)
set -o pipefail
tag=${1:-hp}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 200 python3 bench.py --no-cpu > $out/bench.json || exit 1
python3 -c "import json;d=json.load(open('$out/bench.json'));print('value %.4g gpu_ms %.3f frac %.4f'%(d['value'],d['roofline']['gpu_ms_per_step'],d['roofline']['frac']))"
bash tools/prof_bench.sh $tag --no-cpu --steps 5 --warmup 1 || exit 1
python3 tools/kstats.py gpurun_out/prof_$tag/run_kernel_stats.csv | grep -E 'k_(classify|rs64|scan|runs|flows|results|hs_|hot_)'
bash tools/pmc_bench.sh $tag --no-cpu --steps 5 --warmup 1 || exit 1
grep -A3 -E '^k_(classify_hot|hot_scatter|hot_results|results)' gpurun_out/pmc_$tag/summary.txt | head -40
tail -1 gpurun_out/pmc_$tag/summary.txt
