# round-5 final: GPU suite, smoke, the bench lines (driver flags), rocprofv3 kernel trace of the default bench
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5z_tests.txt 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r5z_tests.txt; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5z_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r5z_bench_c2.json 2> gpurun_out/r5z_bench_c2.err || exit 1
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/r5z_bench_$w.json 2> gpurun_out/r5z_bench_$w.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z_prof -o run -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r5z_prof_bench.json 2> $R/gpurun_out/r5z_prof.err || exit 1
cd $R && python tools/prof_tail.py gpurun_out/r5z_prof 20 > gpurun_out/r5z_prof_tail.csv
