# the driver's bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) and a rocprofv3 trace of it
cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
TAG=${1:-drv}
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -5 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { tail $OUT/prof_$TAG.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/prof_tail.py $OUT/prof_$TAG 20 > $OUT/prof_tail_$TAG.csv && cat $OUT/prof_tail_$TAG.csv
