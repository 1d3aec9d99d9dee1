#!/bin/bash
# Round 5, step A (GPU box): packed entry + 4-byte key table -- parity, bench A/B, trace, cold-kernel phase knobs.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05a}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_packed_device_gpu.py \
  tests/test_cluster_parity_gpu.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; grep -q "Fatal\|core dumped\|Aborted" $out/pytest.log && exit 1; }
tail -3 $out/pytest.log
for rep in 1 2; do
  for envs in "SGA_BENCH_UNPACKED=0" "SGA_BENCH_UNPACKED=1"; do
    extra="--no-parity"; [ $rep = 1 ] && [ "$envs" = "SGA_BENCH_UNPACKED=0" ] && extra=""
    env $envs timeout -k 10 300 python3 bench.py --no-cpu --no-e2e $extra > $out/ab_${envs#*=}_$rep.json 2> $out/ab_${envs#*=}_$rep.err || { tail -5 $out/ab_${envs#*=}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/ab_${envs#*=}_$rep.json').read().strip().splitlines()[-1]); print('[$envs] ms %.4f gpu_ms %.4f' % (d['ms_per_step'], d['roofline']['gpu_ms_per_step']), d.get('parity_sample'))"
  done
done
i=0
for cfg in "SGA_FZ_DEBUG=0" "SGA_FZ_DEBUG=1" "SGA_FZ_DEBUG=2" "SGA_FZ_DEBUG=128" "SGA_HOT_OVERLAP=0"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05a_$i -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --no-parity --steps 10 --warmup 3 > $out/tr_$i.json 2> $out/tr_$i.err || { tail -5 $out/tr_$i.err; exit 1; }
  f=$(find /tmp/r05a_$i -name '*kernel_trace.csv' | head -1)
  cp $f $out/trace_$i.csv
  python3 tools/timeline.py $out/trace_$i.csv > $out/timeline_$i.txt
  echo "== $cfg"; cat $out/timeline_$i.txt
done
