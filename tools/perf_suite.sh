#!/bin/bash
# Kernel timings of the BASELINE configs (device-resident, kernel ms from HIP events):
# C2 rate 16 f32, C4-style rate 8 f32, C3 f64 precision 32, f32 reversible 3D, 128^4 f32 reversible/rate 8.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
LIB=${1:-$R/zfp-par_amd/lib/libzfp.so}
set -e
cd $R
run() { timeout -k 10 120 python tools/kprof.py --lib $LIB "$@" 2>/dev/null; }
run --iters 8 --decode
run --iters 8 --param 8 --decode
run --iters 6 --mode precision --param 32 --dtype f64 --decode
run --iters 6 --mode reversible --decode
run --iters 6 --dims 4 --n 128 --mode reversible --decode
run --iters 6 --dims 4 --n 128 --param 8 --decode
