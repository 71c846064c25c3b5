# final build: GPU suite, smoke, C5 and C2 bench lines
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5t_tests.txt 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r5t_tests.txt; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5t_smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --workload c5 > gpurun_out/r5t_bench_c5.json 2> gpurun_out/r5t_bench_c5.err || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r5t_bench_c2.json 2> gpurun_out/r5t_bench_c2.err
