#!/bin/bash
# Usage (GPU box): bash tools/r04_round.sh <tag> -- the round's record: the whole -m gpu suite (verbose log), smoke,
# the C3 bench line, and every configuration line (bench.py --config c1|c2|c4|c4full|c5a|c5b).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04r}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log
[ $rc = 0 ] || { grep -E "FAILED|ERROR|Error" $out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python3 bench.py > $out/bench_n1.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench_n1.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print('C3 value %.4g ms %.4f frac %.4f cpu %.4g (shard %.4g contended %.4g) e2e %.4g' % (d['value'], d['ms_per_step'], d['roofline']['frac'], c['value'], c['value_shard_parallel'], c['value_contended'], d['end_to_end_host_buffers']['value']))"
for c in c1 c2 c4 c4full c5a c5b; do
  timeout -k 10 500 python3 bench.py --config $c > $out/config_$c.json 2> $out/config_$c.err || { echo "config $c failed"; tail -8 $out/config_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/config_$c.json').read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print('$c', '%.4g' % d['value'], d['unit'], 'ms %.3f' % d['ms_per_step'], 'cpu %.4g' % (c.get('value') or 0), 'parity', d.get('parity_sample'))" | cut -c1-250
done
