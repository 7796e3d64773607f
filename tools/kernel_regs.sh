#!/bin/bash
# VGPRs / spills / occupancy per kernel of one .hip file: bash tools/kernel_regs.sh FILE.hip [FILTER]
f=$1; flt=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o /tmp/_kr.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re,sys
cur=None; rows=[]
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur={'n':m.group(1)}; rows.append(cur); continue
    m=re.search(r'remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)',l)
    if m and cur is not None: cur[m.group(1)]=m.group(2)
for r in rows:
    if re.search(sys.argv[1], r['n']):
        print(f\"{r['n'][:90]:90s} v={r.get('VGPRs')} a={r.get('AGPRs')} vsp={r.get('VGPRs Spill')} ssp={r.get('SGPRs Spill')} scr={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}\")
" "$flt"
