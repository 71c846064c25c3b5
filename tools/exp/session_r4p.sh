# round-4 session p: 4D tests with short reversible slots by default, C5 bench line
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_codec4.py tests/test_gpu_pipeline.py tests/test_gpu_scan.py tests/test_gpu_golden.py > gpurun_out/r4p_tests.txt 2>&1 || { tail -40 gpurun_out/r4p_tests.txt; exit 1; }
tail -2 gpurun_out/r4p_tests.txt
timeout -k 10 300 python bench.py --no-cpu --workload c5 > gpurun_out/r4p_bench_c5.json 2> gpurun_out/r4p_bench_c5.err || exit 1
cat gpurun_out/r4p_bench_c5.json
