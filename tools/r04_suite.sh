#!/bin/bash
# Usage (GPU box): bash tools/r04_suite.sh <tag> -- the whole -m gpu suite (verbose log) and smoke.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04suite}
mkdir -p $out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log
[ $rc = 0 ] || { grep -E "FAILED|ERROR|Error" $out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
