# kernel traces (CSV) of the c3, c4 and c5 bench lines on the final build: per-kernel averages of the last dispatches
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
for w in c3 c4 c5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5p5_$w -o run -- python3 $R/bench.py --workload $w --no-cpu > $R/gpurun_out/r5p5_bench_$w.json 2> $R/gpurun_out/r5p5_$w.err || exit 1
  (cd $R && python tools/prof_tail.py gpurun_out/r5p5_$w 5 > gpurun_out/r5p5_tail_$w.csv) || exit 1
done
