#!/bin/bash
# Builds the engine library of git revision <rev> as sentinel_amd/libsentinel_amd_<name>.so (A/B against the
# working tree with SGA_LIB_VARIANT=<name>).  Usage: bash tools/build_variant.sh <rev> <name>
set -euo pipefail
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/sgavar.XXXX)
git -C "$root" archive "$rev" sentinel_amd/csrc include | tar -x -C "$tmp"
make -s -j8 -C "$tmp/sentinel_amd/csrc" OUT="$root/sentinel_amd/libsentinel_amd_$name.so" "$root/sentinel_amd/libsentinel_amd_$name.so"
rm -rf "$tmp"
echo "built sentinel_amd/libsentinel_amd_$name.so from $rev"
