#!/bin/bash
# 4D iteration: 4D parity tests, then 4D kernel timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-4d}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec4.py tests/test_gpu_types.py tests/test_gpu_scan.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
{
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 --sha --decode &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode precision --param 16 --iters 5 --sha &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode rate --param 8 --iters 5 --sha
} > $OUT/kprof_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/kprof_$TAG.log; exit $rc
