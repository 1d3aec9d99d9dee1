#!/bin/bash
# Builds the engine library of git revision <rev> as sentinel_amd/libsentinel_amd_<name>.so (A/B against the
# working tree with SGA_LIB_VARIANT=<name>).  Usage: bash tools/build_variant.sh <rev> <name> [extra compiler flags]
# (<rev> WORKTREE: the working tree's sources)
set -euo pipefail
rev=$1; name=$2; extra=${3:-}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/sgavar.XXXX)
if [ "$rev" = WORKTREE ]; then
    mkdir -p "$tmp/sentinel_amd"
    cp -r "$root/sentinel_amd/csrc" "$tmp/sentinel_amd/" && rm -rf "$tmp/sentinel_amd/csrc/build"
    cp -r "$root/include" "$tmp/"
else
    git -C "$root" archive "$rev" sentinel_amd/csrc include | tar -x -C "$tmp"
fi
make -s -j8 -C "$tmp/sentinel_amd/csrc" EXTRA="$extra" OUT="$root/sentinel_amd/libsentinel_amd_$name.so" "$root/sentinel_amd/libsentinel_amd_$name.so"
rm -rf "$tmp"
echo "built sentinel_amd/libsentinel_amd_$name.so from $rev"
