#!/bin/bash
# usage: regs.sh file.hip [extra flags]; prints vgpr/sgpr/lds/scratch of render kernels
f=$1; shift
b=$(basename $f .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fno-gpu-rdc -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None --cuda-device-only -S -o /tmp/$b.s $f "$@" 2>/dev/null
python3 - /tmp/$b.s <<'PY'
import re,sys
s=open(sys.argv[1]).read()
for blk in s.split('  - .agpr_count:')[1:]:
    name=re.search(r'\.name:\s+(\S+)',blk).group(1)
    if re.search(r'render|tile_cut|sum_records|preprocess', name):
        g=lambda k: re.search(r'\.'+k+r':\s+(\d+)',blk).group(1)
        print(name[:60], 'vgpr',g('vgpr_count'),'sgpr',g('sgpr_count'),'lds',g('group_segment_fixed_size'),'scratch',g('private_segment_fixed_size'))
PY
