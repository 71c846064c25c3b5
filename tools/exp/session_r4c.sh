# round-4 session c: 4D tests, C5 bench, rocprofv3 trace + PMC of the C2 bench
set -o pipefail
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_codec4.py tests/test_gpu_scan.py tests/test_kernel_symbols.py > gpurun_out/r4c_tests.txt 2>&1 || { tail -30 gpurun_out/r4c_tests.txt; exit 1; }
tail -1 gpurun_out/r4c_tests.txt
timeout -k 10 300 python bench.py --no-cpu --workload c5 > gpurun_out/r4c_bench_c5.json 2> gpurun_out/r4c_bench_c5.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4c_prof -o run -- python $R/bench.py --no-cpu > $R/gpurun_out/r4c_prof_bench.json 2> $R/gpurun_out/r4c_prof_bench.err || exit 1
cd $R
python tools/prof_tail.py gpurun_out/r4c_prof 20 > gpurun_out/r4c_prof_tail.csv
./tools/pmc_bin.sh r4c_c2 -- python $R/bench.py --no-cpu --steps 3 --warmup 1 --clock-warm-ms 50 > gpurun_out/r4c_pmc.log 2>&1 || exit 1
