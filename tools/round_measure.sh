#!/bin/bash
# Round-end measurements: bench line, rocprofv3 kernel stats of the bench, PMC
# passes of the C2 kernels (one counter group per run).  Writes gpurun_out/*_<tag>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r2}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -5 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python $R/bench.py --steps 10 --warmup 5 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
bash $R/tools/pmc_round.sh $TAG || exit 1
python $R/tools/pmc_summary.py $OUT/pmc_$TAG > $OUT/pmc_$TAG.txt && echo pmc ok
