#!/bin/bash
# Usage (on the GPU box): bash tools_prof.sh <tag> [bench args...]
# rocprofv3 kernel-trace summary of a bench run; keeps only the stats CSVs.
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$tag -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_$tag/bench.out 2>&1
rc=$?
find /tmp/prof_$tag -name "*stats*" -exec cp {} gpurun_out/prof_$tag/ \;
exit $rc
