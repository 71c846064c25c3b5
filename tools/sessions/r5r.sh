# product build with the one-window 4D loop, the f64 short-slot decoder changes and plausible scan starts:
# full GPU suite, C5/C3/C2 against HEAD~ (lib_var/head), the index scan
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5r_tests.txt 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r5r_tests.txt; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for v in lib_var/head lib; do
    for w in c5 c3 c2; do
      ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload $w --steps 8 --warmup 3 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v $w enc', d['roofline']['kernel_ms'], 'dec', d.get('decode_kernel_ms'))" >> gpurun_out/r5r_ab.txt || exit 1
    done
  done
done
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 2 > gpurun_out/r5r_scan.txt 2>&1 || exit 1
timeout -k 10 300 python tools/scan_bench.py --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 2 >> gpurun_out/r5r_scan.txt 2>&1
