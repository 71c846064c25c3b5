#!/bin/bash
# Tabulate per-kernel VGPR/SGPR/scratch/occupancy for the HIP library (gfx950).
cd "$(dirname "$0")/../zfp-par_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -Icsrc/host -Icsrc/hip \
  -c --cuda-device-only -Rpass-analysis=kernel-resource-usage csrc/hip/zfp_hip.hip -o /tmp/kres.o "$@" 2>&1 |
python3 -c '
import re,sys
cur=None; rows={}
for line in sys.stdin:
    m=re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\S+)",line)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name": cur=v; rows[cur]={}
    else: rows[cur][k]=v
for f,r in rows.items():
    print("%-70s vgpr=%-4s sgpr=%-4s scratch=%-5s occ=%-2s vspill=%s sspill=%s"%(f[:70],r.get("VGPRs"),r.get("SGPRs"),r.get("ScratchSize [bytes/lane]"),r.get("Occupancy [waves/SIMD]"),r.get("VGPRs Spill"),r.get("SGPRs Spill")))
'
