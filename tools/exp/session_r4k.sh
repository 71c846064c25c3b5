# round-4 session k: block API parity on the GPU, zfpy/zfp_parallel tests, zfp_parallel throughput
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_block_api.py tests/test_zfpy.py tests/test_zfpy_golden.py tests/test_gpu_pool.py > gpurun_out/r4k_tests.txt 2>&1 || { tail -40 gpurun_out/r4k_tests.txt; exit 1; }
tail -2 gpurun_out/r4k_tests.txt
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 --profile > gpurun_out/r4k_zpar.txt 2>&1 || exit 1
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 --threads 4 >> gpurun_out/r4k_zpar.txt 2>&1 || exit 1
cat gpurun_out/r4k_zpar.txt
