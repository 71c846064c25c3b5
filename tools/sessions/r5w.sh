# index scan: candidate-check budget of 64 Kbit per segment (lib_var/scancap) against the product (unbounded)
mkdir -p gpurun_out
for v in lib lib_var/scancap lib lib_var/scancap; do
  echo "== $v" >> gpurun_out/r5w_scan.txt
  ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --lib zfp-par_amd/$v/libzfp.so --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 >> gpurun_out/r5w_scan.txt 2>&1 || exit 1
done
for v in lib lib_var/scancap; do
  echo "== $v f64" >> gpurun_out/r5w_scan.txt
  timeout -k 10 300 python tools/scan_bench.py --lib zfp-par_amd/$v/libzfp.so --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 2 >> gpurun_out/r5w_scan.txt 2>&1 || exit 1
done
