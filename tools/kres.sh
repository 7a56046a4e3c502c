#!/bin/bash
# Per-kernel VGPR / scratch / LDS of a built object (code-object metadata), filtered by a name
# pattern.  Usage: tools/kres.sh custom-k8s-scheduler_amd/build/qs_kernels.o k_la_stream_res
set -e
obj=$1; pat=${2:-k_}
tmp=$(mktemp -d)
/opt/rocm/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fat.bin "$obj"
/opt/rocm/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/k.co
/opt/rocm/llvm/bin/llvm-readelf --notes $tmp/k.co | python3 -c "
import sys, re
txt = sys.stdin.read()
for blk in re.split(r'\n\s+- \.agpr_count', txt)[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk).group(1)
    if '$pat' not in name: continue
    g = lambda k: re.search(r'\.' + k + r':\s+(\d+)', blk).group(1)
    short = re.search(r'(k_\w+?)I(\w+?)EEEv', name)
    print(short.group(1) if short else name[:50], short.group(2) if short else '', 'vgpr', g('vgpr_count'), 'sgpr', g('sgpr_count'),
          'scratch', g('private_segment_fixed_size'), 'lds', g('group_segment_fixed_size'))
"
rm -rf $tmp
