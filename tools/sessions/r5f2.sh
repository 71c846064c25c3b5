# final lines on the final build: the four workloads (driver flags) and the kernel trace (CSV) of the default bench
mkdir -p gpurun_out
R=$PWD
for w in c2 c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/r5f2_bench_$w.json 2> gpurun_out/r5f2_bench_$w.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5f2_prof -o run -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r5f2_prof_bench.json 2> $R/gpurun_out/r5f2_prof.err || exit 1
cd $R && python tools/prof_tail.py gpurun_out/r5f2_prof 20 > gpurun_out/r5f2_prof_tail.csv
