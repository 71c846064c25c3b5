# A/B: look-back aggregate from a length pre-pass (lib_var/prepass) against the product (lib), C5 chunk and 128^4
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in lib lib_var/prepass; do
    ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v c5 enc', d['roofline']['kernel_ms'], 'dec', d['decode_kernel_ms'], d['lossless_roundtrip'])" >> gpurun_out/r5o_ab.txt || exit 1
  done
done
timeout -k 10 300 bash tools/ab_lib.sh "--iters 6 --dims 4 --n 128 --mode reversible" lib lib_var/prepass >> gpurun_out/r5o_ab.txt 2>&1  # stream sha256 must match
