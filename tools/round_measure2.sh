#!/bin/bash
# Round-end measurements (round 2, second session): 4D parity tests, bench
# line, rocprofv3 kernel stats of the bench, PMC passes of C2, C3 and C5-mode
# kernels, kernel timings of every config.  Writes gpurun_out/*_<tag>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r2d}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec4.py tests/test_gpu_pipeline.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests4_$TAG.log 2>&1 || { echo tests failed; tail -20 $OUT/tests4_$TAG.log; exit 1; }
tail -2 $OUT/tests4_$TAG.log
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail -5 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
{
timeout -k 10 120 python tools/kprof.py --mode rate --param 16 --iters 12 --decode &&
timeout -k 10 120 python tools/kprof.py --mode precision --param 32 --dtype f64 --iters 6 --decode &&
timeout -k 10 120 python tools/kprof.py --mode reversible --iters 6 --decode &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 --decode &&
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode rate --param 8 --iters 5 --decode
} > $OUT/kprof_$TAG.txt 2>&1 || { echo kprof failed; tail $OUT/kprof_$TAG.txt; exit 1; }
grep -v amdgpu.ids $OUT/kprof_$TAG.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python $R/bench.py --steps 20 --warmup 10 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { echo prof failed; exit 1; }
echo prof ok
python $R/tools/prof_tail.py $OUT/prof_$TAG 20 > $OUT/prof_tail_$TAG.csv && cat $OUT/prof_tail_$TAG.csv
bash $R/tools/pmc_round.sh ${TAG}_c2 --mode rate --param 16 --decode || exit 1
bash $R/tools/pmc_round.sh ${TAG}_c3 --mode precision --param 32 --dtype f64 --decode || exit 1
bash $R/tools/pmc_round.sh ${TAG}_c5 --dims 4 --n 128 --mode reversible --decode || exit 1
for k in c2 c3 c5; do python $R/tools/pmc_summary.py $OUT/pmc_${TAG}_$k > $OUT/pmc_${TAG}_$k.txt; done
echo pmc ok
