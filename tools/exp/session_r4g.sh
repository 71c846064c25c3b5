# round-4 session g: where the f64 short-slot decoder's length check costs (variants), zfp_parallel with direct bytes targets
set -o pipefail
for v in vm2 cur vx3 vx5 vm2 cur vx3 vx5; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f64 --mode precision --param 32 --iters 4 --decode 2>&1 | grep decode || exit 1
done > gpurun_out/r4g_verify_ab.txt
cat gpurun_out/r4g_verify_ab.txt
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 --profile > gpurun_out/r4g_zpar.txt 2>&1 || exit 1
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 --threads 4 >> gpurun_out/r4g_zpar.txt 2>&1 || exit 1
cat gpurun_out/r4g_zpar.txt
