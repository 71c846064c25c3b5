mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5e_tests.txt 2>&1; echo "tests rc=$?" >> gpurun_out/r5e_tests.txt
ZFP_HIP_TRACE4=1 ZFP_BENCH_LIB=zfp-par_amd/lib_var/trace/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --clock-warm-ms 0 > gpurun_out/r5e_trace.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/r5e_c5.json 2>&1 || exit 1
ZFP_BENCH_LIB=zfp-par_amd/lib_var/nohalf/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/r5e_c5_nohalf.json 2>&1 || exit 1
timeout -k 10 300 bash tools/perf_suite.sh > gpurun_out/r5e_perf.txt 2>&1 || exit 1
timeout -k 10 120 python tools/block_api_latency.py > gpurun_out/r5e_blockapi.txt 2>&1
