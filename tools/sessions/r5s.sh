# index scan with phase-A refusals (lib_var/scan2); C3 decode variants (pin / scalar wave index) against HEAD~ and the product
mkdir -p gpurun_out
L=zfp-par_amd/lib_var/scan2/libzfp.so
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 2 > gpurun_out/r5s_scan.txt 2>&1 || exit 1
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --lib $L --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 2 >> gpurun_out/r5s_scan.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in lib_var/head lib lib_var/c3np lib_var/c3vw; do
    ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c3 enc', d['roofline']['kernel_ms'], 'dec', d.get('decode_kernel_ms'))" >> gpurun_out/r5s_ab.txt || exit 1
  done
done
