# decode4 overflow waves from whole segments (lib_var/ovfpk) against padded slots (lib): C5 chunk, 3 reps
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in lib lib_var/ovfpk; do
    ZFP_HIP_VERBOSE=1 ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu 2>gpurun_out/r5u_err.txt | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c5 enc', d['roofline']['kernel_ms'], 'dec', d['decode_kernel_ms'], d['lossless_roundtrip'])" >> gpurun_out/r5u_ab.txt || exit 1
  done
done
grep decode4 gpurun_out/r5u_err.txt | tail -2 >> gpurun_out/r5u_ab.txt
