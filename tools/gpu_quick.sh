#!/bin/bash
# Iteration loop on the GPU box: parity tests (stop at first failure), then the
# light kernel timer.  Every GPU step has its own limit; the chain ends at the
# first non-zero exit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-q}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 $OUT/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kprof.py --iters 5 --decode > $OUT/kprof_$TAG.log 2>&1
rc=$?; cat $OUT/kprof_$TAG.log; exit $rc
