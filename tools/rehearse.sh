#!/bin/bash
# Usage (GPU box): bash tools/rehearse.sh <tag> -- the N-rank paths on one GPU (SGA_BENCH_ONE_DEVICE=1: both ranks
# on device 0, the per-second gather over gloo) for C3 and C2, beside the one-rank lines of the same code.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-reh}
mkdir -p $out
run() {  # name, env, args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 900 python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "FAIL $name"; tail -5 $out/$name.err; exit 1; }
  python3 - "$out/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("metric_allgather") or {}
print(sys.argv[2], "n_gpus", d["n_gpus"], "ms %.3f" % d["ms_per_step"], "value %.4g" % d["value"],
      "group_size", m.get("group_size"), "parity", json.dumps(d.get("parity_sample"))[:160])
PY
}
run c3_gpus2 "SGA_BENCH_ONE_DEVICE=1" --gpus 2 --no-cpu --no-e2e
run c2_gpus2 "SGA_BENCH_ONE_DEVICE=1" --config c2 --gpus 2
run c3_gpus1 "SGA_NONE=0" --no-cpu --no-e2e
run c3_nometric "SGA_BENCH_METRIC_EVERY=100000" --no-cpu --no-e2e --no-parity
