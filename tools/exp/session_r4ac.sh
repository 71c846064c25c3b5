# round-4 session ac: zfpy GPU tests with fixed-rate streams written straight into bytes; zfp_parallel throughput
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_zfpy.py tests/test_zfpy_golden.py tests/test_gpu_pool.py tests/test_gpu_distributed.py tests/test_cli.py > gpurun_out/r4ac_tests.txt 2>&1 || { tail -30 gpurun_out/r4ac_tests.txt; exit 1; }
tail -1 gpurun_out/r4ac_tests.txt
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 > gpurun_out/r4ac_zpar.txt 2>&1 || exit 1
cat gpurun_out/r4ac_zpar.txt | grep zfp_parallel
