#!/bin/bash
# Bench (c2 default and c4), rocprofv3 kernel trace + stats of the c2 bench
# command, and the tail average of the timed steps (tools/prof_tail.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r2e}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -5 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 400 python bench.py --workload c4 --steps 10 --warmup 5 --no-cpu > $OUT/bench_c4_$TAG.json 2> $OUT/bench_c4_$TAG.err || { echo bench c4 failed; tail -5 $OUT/bench_c4_$TAG.err; exit 1; }
cat $OUT/bench_c4_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python $R/bench.py --steps 20 --warmup 10 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { echo prof failed; exit 1; }
tail -1 $OUT/prof_$TAG.log
python $R/tools/prof_tail.py $OUT/prof_$TAG 20 > $OUT/prof_tail_$TAG.csv && cat $OUT/prof_tail_$TAG.csv
