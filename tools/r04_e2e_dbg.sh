#!/bin/bash
# Usage (GPU box): bash tools/r04_e2e_dbg.sh <tag> -- the host-buffer pipeline's parity test, then its phase
# times (SGA_PIPE_DEBUG) inside the C3 bench's end-to-end leg.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04e2}
mkdir -p $out
timeout -k 10 200 python3 -u -m pytest tests/test_cluster_parity_gpu.py -m gpu -x -q -k host_batches --timeout 150 \
    --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
SGA_PIPE_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
grep "^pipe" $out/bench.err | tail -3
python3 -c "
import json; d=json.load(open('$out/bench.json')); e=d.get('end_to_end_host_buffers'); print('e2e', e['value'], e['ms_per_batch'])"
timeout -k 10 300 python3 -u -m pytest tests/test_param_args_gpu.py -m gpu -x -q -k "many_indices" --timeout 250 \
    --timeout-method thread > $out/pytest_idx.log 2>&1 || { tail -30 $out/pytest_idx.log; exit 1; }
tail -1 $out/pytest_idx.log
