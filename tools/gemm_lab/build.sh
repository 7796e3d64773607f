#!/bin/bash
# Build the GEMM lab library (tuning only): bash tools/gemm_lab/build.sh
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared f16lab.hip -o libf16lab.so \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re,sys
cur=None; rows=[]
for l in sys.stdin:
    if 'error' in l: print(l.rstrip())
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur={'n':m.group(1)}; rows.append(cur); continue
    m=re.search(r'remark:\s+(VGPRs|AGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)',l)
    if m and cur is not None: cur[m.group(1)]=m.group(2)
for r in rows:
    print(f\"{r['n'][:60]:60s} v={r.get('VGPRs')} a={r.get('AGPRs')} spill={r.get('VGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}\")
"
