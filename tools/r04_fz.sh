#!/bin/bash
# Usage (GPU box): bash tools/r04_fz.sh <tag> -- k_cold_fused phase times (SGA_FZ_DEBUG=16: in-kernel
# wall_clock64 marks per workgroup, one stream) and the C3 bench line, for an A/B of the cold stage.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04fz}
out=gpurun_out/$tag
mkdir -p $out
SGA_FZ_DEBUG=16 timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 4 --warmup 1 > $out/fz.json 2> $out/fz.err || { tail -20 $out/fz.err; exit 1; }
grep "fz phases" $out/fz.err | tail -3
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))"
