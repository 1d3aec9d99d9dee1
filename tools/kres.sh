#!/bin/bash
# Usage: bash tools/kres.sh [pattern]  -- VGPR / LDS / spill per kernel of the built cluster object
set -e
o=${2:-/root/repo/sentinel_amd/csrc/build/cluster.o}
d=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$d/fat.bin $o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $d/k.co > $d/notes.txt
python3 - "$d/notes.txt" "${1:-.}" <<'PY'
import re,sys
t=open(sys.argv[1]).read()
for blk in t.split('- .agpr_count')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk).group(1)
    if not re.search(sys.argv[2], name): continue
    g=lambda k: re.search(r'\.'+k+r':\s+(\d+)',blk).group(1)
    print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} spill {g('vgpr_spill_count')}")
PY
rm -rf $d
