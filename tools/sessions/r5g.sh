mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec4.py tests/test_gpu_arrays.py -q --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.txt 2>&1; echo "tests rc=$?" >> gpurun_out/r5g_tests.txt
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/r5g_c5.json 2>&1 || exit 1
ZFP_HIP_TRACE4=1 ZFP_BENCH_LIB=zfp-par_amd/lib_var/trace/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --clock-warm-ms 0 > gpurun_out/r5g_trace.txt 2>&1 || exit 1
