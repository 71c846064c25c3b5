#!/bin/bash
# Full GPU parity suite, then kernel timings: C2 (rate 16 f32), C3 (f64
# precision 32) with short and full-size slots, C5-mode 4D reversible.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-full}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
{
timeout -k 10 120 python tools/kprof.py --mode rate --param 16 --iters 12 --sha --decode &&
timeout -k 10 120 python tools/kprof.py --mode precision --param 32 --dtype f64 --iters 6 --sha --decode &&
ZFP_HIP_FULL_SLOTS=1 timeout -k 10 120 python tools/kprof.py --mode precision --param 32 --dtype f64 --iters 6 --sha --decode &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 4 --sha --decode &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode rate --param 8 --iters 4 --sha --decode
} > $OUT/kprof_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/kprof_$TAG.log; exit $rc
