#!/bin/bash
# Quick GPU iteration: cluster parity tests, headline bench, rocprofv3 kernel stats.
# Usage (GPU box): bash tools/r02_quick.sh <tag> [pytest target]
set -o pipefail
tag=${1:-q}
tgt=${2:-tests/test_cluster_parity_gpu.py}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest $tgt -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -4 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/bench.json'));r=d['roofline'];print('value %.3e ms/step %.3f gpu_ms %.3f frac %.3f path %s'%(d['value'],d['ms_per_step'],r['gpu_ms_per_step'],r['frac'],d.get('last_batch_path')))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu > $out/prof_bench.json 2> $out/prof.err || { tail -5 $out/prof.err; exit 1; }
find /tmp/prof_$tag -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
find /tmp/prof_$tag -name "*kernel_trace.csv" -exec cp {} $out/kernel_trace.csv \;
python3 tools/ktrace.py $out/kernel_trace.csv --last 10 | grep -v "k_hist \|k_emit\|k_flags\|k_scan\|at::native\|rocclr\|k_init_slots\|k_conc_reset\|k_hot_reset" | head -40
