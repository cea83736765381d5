#!/bin/bash
# kres.sh <object.o> [name-filter]: VGPR / SGPR / spill / scratch of each gfx950 kernel in a hipcc object. Dev tool.
set -e
O=$1; F=${2:-.}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$O"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c "
import re,sys
t=sys.stdin.read()
# metadata fields are alphabetical: .group_segment_fixed_size precedes .name, the rest follow it
parts=t.split('.name:')
for i,b in enumerate(parts[1:]):
    n=b.split('\n')[0].strip()
    prev=parts[i]
    if not re.search(sys.argv[1], n): continue
    g=lambda k: (re.search(r'\.'+k+r':\s+(\d+)',b) or [None,'-'])[1]
    print('vgpr',g('vgpr_count'),'sgpr',g('sgpr_count'),'vspill',g('vgpr_spill_count'),'scratch',g('private_segment_fixed_size'),'lds',(re.findall(r'\.group_segment_fixed_size:\s+(\d+)',prev) or ['-'])[-1],n[:150])
" "$F"
rm -rf $T
