# round-4 final B: bench lines (driver flags), rocprofv3 trace of the default bench, HBM traffic of the c3/c4/c5 kernels
set -o pipefail
R=$PWD
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r4z_bench_c2.json 2> gpurun_out/r4z_bench_c2.err || exit 1
cat gpurun_out/r4z_bench_c2.json
for w in c3 c4 c5; do
  timeout -k 10 300 python bench.py --no-cpu --workload $w > gpurun_out/r4z_bench_$w.json 2> gpurun_out/r4z_bench_$w.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4z_prof -o run -- python $R/bench.py --no-cpu > $R/gpurun_out/r4z_prof_bench.json 2> $R/gpurun_out/r4z_prof_bench.err || exit 1
cd $R
python tools/prof_tail.py gpurun_out/r4z_prof 20 > gpurun_out/r4z_prof_tail.csv || exit 1
for w in c4 c5; do
  ./tools/pmc_traffic.sh r4z_$w -- python $R/bench.py --no-cpu --workload $w --steps 2 --warmup 1 --clock-warm-ms 50 > gpurun_out/r4z_pmc_$w.log 2>&1 || exit 1
done
cat gpurun_out/r4z_prof_tail.csv
