# A/B: negabinary XOR folded into the decoders' last transpose step (lib_var/dnb) against the product build
mkdir -p gpurun_out
o=gpurun_out/r5dn_ab.txt
: > $o
for rep in 1 2; do
  for v in lib lib_var/dnb; do
    for w in c2 c3; do
      ZFP_BENCH_LIB=zfp-par_amd/$v/libzfp.so timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v $w enc', d['roofline']['kernel_ms'], 'dec', d.get('decode_kernel_ms'), d.get('decode_max_abs_err'))" >> $o || exit 1
    done
  done
done
