#!/bin/bash
# Index-scan time against the segment length (ZFP_HIP_SCAN_SEG_BITS).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
for L in "" 65536 262144 1048576; do
  echo "== L=${L:-default}"
  if [ -n "$L" ]; then export ZFP_HIP_SCAN_SEG_BITS=$L; else unset ZFP_HIP_SCAN_SEG_BITS; fi
  timeout -k 10 200 python tools/scan_bench.py --n 512 --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
done
