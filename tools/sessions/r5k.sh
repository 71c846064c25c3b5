# decode4 phase trace on the C5 chunk (trace build), then the product C5 line
mkdir -p gpurun_out
ZFP_HIP_TRACE4=1 ZFP_BENCH_LIB=zfp-par_amd/lib_var/trace/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --clock-warm-ms 0 > gpurun_out/r5k_trace.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/r5k_c5.json 2>&1
