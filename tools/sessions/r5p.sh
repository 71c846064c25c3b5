# index scan: plausible chain starts in pass 1 (lib_var/scanpl) vs segment-start chains (ZFP_HIP_SCAN_PLAUSIBLE=0)
mkdir -p gpurun_out
L=zfp-par_amd/lib_var/scanpl/libzfp.so
for pl in 1 0; do
  echo "== plausible=$pl 128^4 f32 reversible" >> gpurun_out/r5p_scan.txt
  ZFP_HIP_SCAN_PLAUSIBLE=$pl ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 2 >> gpurun_out/r5p_scan.txt 2>&1 || exit 1
  echo "== plausible=$pl 512^3 f64 precision 32" >> gpurun_out/r5p_scan.txt
  ZFP_HIP_SCAN_PLAUSIBLE=$pl ZFP_HIP_SCAN_TRACE=1 timeout -k 10 300 python tools/scan_bench.py --lib $L --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 2 >> gpurun_out/r5p_scan.txt 2>&1 || exit 1
done
