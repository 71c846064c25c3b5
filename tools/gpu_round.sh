#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Every GPU step
# has its own time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
echo "tests exit=$?" ; tail -3 $OUT/tests_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && \
  echo "bench ok" && cat $OUT/bench_$TAG.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/prof_$TAG.log 2>&1 && echo "prof ok" && \
find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -3
