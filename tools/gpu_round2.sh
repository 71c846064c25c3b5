#!/bin/bash
# One GPU session for a profile round: bench (+CPU baseline), rocprofv3 kernel
# stats of the same bench, and kernel timings of the other BASELINE configs
# (C3 f64 precision 32, C5-like 4D reversible) through tools/kprof.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
echo "bench ok"; cat $OUT/bench_$TAG.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_$TAG.log 2>&1) || exit 1
echo "prof ok"
{
timeout -k 10 120 python tools/kprof.py --mode rate --param 16 --iters 4 --decode &&
timeout -k 10 120 python tools/kprof.py --mode precision --param 32 --dtype f64 --iters 4 --decode &&
timeout -k 10 120 python tools/kprof.py --mode reversible --iters 4 --decode &&
timeout -k 10 300 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 3 --decode &&
timeout -k 10 300 python tools/kprof.py --dims 4 --n 128 --mode rate --param 8 --iters 3 --decode
} > $OUT/kprof_$TAG.txt 2>&1
echo "kprof rc=$?"; grep -v amdgpu.ids $OUT/kprof_$TAG.txt
