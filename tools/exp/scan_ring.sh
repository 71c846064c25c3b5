#!/bin/bash
# Index-scan time of ring-size variants (lib_var/ring32, ring64: ZFP_SCAN_RING_WORDS)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
for v in lib lib_var/ring32 lib_var/ring64; do
  for cfg in "65536:0" "131072:524288"; do
    export ZFP_HIP_SCAN_SEG_BITS=${cfg%%:*} ZFP_HIP_SCAN_LEAD_BITS=${cfg##*:}
    echo "== $v L=$ZFP_HIP_SCAN_SEG_BITS lead=$ZFP_HIP_SCAN_LEAD_BITS"
    L=zfp-par_amd/$v/libzfp.so
    timeout -k 10 200 python tools/scan_bench.py --lib $L --n 512 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
    timeout -k 10 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
