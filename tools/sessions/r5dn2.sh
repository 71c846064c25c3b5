# product build with the folded negabinary decode: GPU suite, smoke, C2 bench line
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5dn2_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r5dn2_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r5dn2_bench_c2.json 2> gpurun_out/r5dn2_bench_c2.err || exit 1
