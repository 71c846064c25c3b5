# closed-form 4D plane parser: 4D/scan GPU tests, C5 bench, A/B decode against HEAD~ build
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec4.py tests/test_gpu_scan.py tests/test_gpu_arrays.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5l_tests.txt 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r5l_tests.txt; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for v in lib_var/head lib; do
    ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'enc', d['roofline']['kernel_ms'], 'dec', d['decode_kernel_ms'], d['lossless_roundtrip'])" >> gpurun_out/r5l_ab.txt || exit 1
  done
done
timeout -k 10 300 bash tools/ab_lib.sh "--iters 6 --dims 4 --n 128 --mode reversible --decode" lib_var/head lib >> gpurun_out/r5l_ab.txt 2>&1
ZFP_HIP_TRACE4=1 ZFP_BENCH_LIB=zfp-par_amd/lib_var/trace/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --clock-warm-ms 0 > gpurun_out/r5l_trace.txt 2>&1
