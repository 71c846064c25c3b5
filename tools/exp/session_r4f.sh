# round-4 session f: index-verification forms A/B on the C3 f64 decoder; zfp_parallel compress under pipeline settings
set -o pipefail
for v in old cur vm1 vm2 cur vm1 vm2; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f64 --mode precision --param 32 --iters 4 --decode 2>&1 | grep decode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f32 --mode reversible --iters 4 --decode 2>&1 | grep decode || exit 1
done > gpurun_out/r4f_verify_ab.txt
cat gpurun_out/r4f_verify_ab.txt
for cfg in "" "ZFP_HIP_NO_PIPE=1" "ZFP_HIP_PIPE_SLAB_MB=64" "ZFP_HIP_PIPE_SLAB_MB=256"; do
  for th in 8 4 2; do
    echo "== $cfg threads $th"
    env $cfg timeout -k 10 120 python tools/zfp_par_bench.py --reps 3 --threads $th 2>&1 | grep zfp_parallel || exit 1
  done
done > gpurun_out/r4f_zpar.txt
cat gpurun_out/r4f_zpar.txt
