#!/bin/bash
# Short-slot / overflow-pool iteration: parity tests of the 3D codec, then
# kernel timings of the variable-rate configs (stream hashes for exactness).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-ovf}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_codec4.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
{
timeout -k 10 120 python tools/kprof.py --mode precision --param 32 --dtype f64 --iters 6 --sha --decode &&
timeout -k 10 120 python tools/kprof.py --mode reversible --iters 6 --sha --decode &&
timeout -k 10 120 python tools/kprof.py --mode precision --param 16 --iters 6 --sha &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 4 --sha --decode
} > $OUT/kprof_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/kprof_$TAG.log; exit $rc
