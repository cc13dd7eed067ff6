#!/bin/bash
# Per-kernel VGPR/SGPR/scratch/occupancy of spt_kernels.hip (hipcc -Rpass-analysis).
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -ffp-contract=off -std=c++17 --offload-arch=gfx950 -Iinclude -Isoftware-path-tracer_amd/csrc \
  ${EXTRA:-} -c software-path-tracer_amd/csrc/spt_kernels.hip -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c "
import re,sys
cur=None; rows={}
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); rows[cur]={}; continue
    for k in ('TotalSGPRs','VGPRs','ScratchSize \[bytes/lane\]','Occupancy \[waves/SIMD\]','LDS Size \[bytes/block\]'):
        m=re.search(k+r': (\d+)',l)
        if m and cur: rows[cur][k.split()[0]]=m.group(1)
for n,r in rows.items():
    print(f\"{n[:60]:60s} sgpr={r.get('TotalSGPRs')} vgpr={r.get('VGPRs')} scratch={r.get('ScratchSize')} occ={r.get('Occupancy')} lds={r.get('LDS')}\")
"
