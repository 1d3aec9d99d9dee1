#!/bin/bash
# Usage (GPU box): bash tools/r04_e2e.sh <tag> -- pipelined host-batch parity tests, the C3 bench line (with the
# end-to-end host-buffer leg), and a kernel trace of C4 full mode (entries vs exits).
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04e}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_cluster_parity_gpu.py -m gpu -x -q -k "host_batches or zipf_c3" \
    --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json')); e=d['extra']['end_to_end_host_buffers'] if 'extra' in d else d.get('end_to_end_host_buffers')
print('C3', d['value'], d['ms_per_step'], 'e2e', e)" || tail -c 800 $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c4full_prof -o c4full -- python3 bench.py --config c4full --steps 1 --warmup 1 --no-cpu > $out/c4full.json 2> $out/c4full.err || { tail -5 $out/c4full.err; exit 1; }
tail -c 300 $out/c4full.json
SGA_BENCH_PIPE=1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $out/bench_pipe.json 2> $out/bench_pipe.err || { tail -5 $out/bench_pipe.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $out/bench_nopipe.json 2> $out/bench_nopipe.err || { tail -5 $out/bench_nopipe.err; exit 1; }
python3 -c "
import json
for k in ('pipe','nopipe'):
    d=json.load(open('$out/bench_%s.json'%k)); print(k, d['value'], d['ms_per_step'])"
