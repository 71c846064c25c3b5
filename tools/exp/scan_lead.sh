#!/bin/bash
# Index-scan time against the segment length and the pass-1 lead-in
# (ZFP_HIP_SCAN_SEG_BITS, ZFP_HIP_SCAN_LEAD_BITS); "" = the library default.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
for cfg in ":" "65536:0" "65536:262144" "65536:524288" "32768:524288" "131072:524288" "131072:1048576"; do
  L=${cfg%%:*}
  D=${cfg##*:}
  echo "== L=${L:-default} lead=${D:-default}"
  if [ -n "$L" ]; then export ZFP_HIP_SCAN_SEG_BITS=$L; else unset ZFP_HIP_SCAN_SEG_BITS; fi
  if [ -n "$D" ]; then export ZFP_HIP_SCAN_LEAD_BITS=$D; else unset ZFP_HIP_SCAN_LEAD_BITS; fi
  timeout -k 10 200 python tools/scan_bench.py --n 512 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
