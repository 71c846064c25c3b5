# A/B: lean 4D group-test loop (lib_var/lean) and the f64 block-position change (lib) against HEAD~ (lib_var/head)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5n_tests.txt 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r5n_tests.txt; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for v in lib_var/head lib lib_var/lean; do
    ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c5 enc', d['roofline']['kernel_ms'], 'dec', d['decode_kernel_ms'], d['lossless_roundtrip'])" >> gpurun_out/r5n_ab.txt || exit 1
  done
  for v in lib_var/head lib; do
    ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c3 enc', d['roofline']['kernel_ms'], 'dec', d.get('decode_kernel_ms'))" >> gpurun_out/r5n_ab.txt || exit 1
  done
done
