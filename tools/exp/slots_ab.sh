#!/bin/bash
# A/B of short vs full-size slots for the variable-rate encoders, plus a
# rocprofv3 kernel-stats pass of the 4D reversible encode (encode4 + patch).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
OUT=$R/gpurun_out
for full in "" 1; do
  echo "== ZFP_HIP_FULL_SLOTS=$full"
  export ZFP_HIP_FULL_SLOTS=$full; [ -z "$full" ] && unset ZFP_HIP_FULL_SLOTS
  timeout -k 10 120 python tools/kprof.py --mode precision --param 16 --iters 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python tools/kprof.py --mode accuracy --param 1e-3 --iters 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode precision --param 16 --iters 5 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode rate --param 8 --iters 5 --sha 2>&1 | grep -v amdgpu.ids || exit 1
done
unset ZFP_HIP_FULL_SLOTS
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof4 -o run -- python $R/tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 > $OUT/prof4.log 2>&1 || exit 1
find $OUT/prof4 -name "*kernel_stats.csv" -exec cat {} \;
