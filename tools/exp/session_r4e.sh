# round-4 session e: C3 f64 decode A/B (round-3 library vs current, stale/scan flags), zfp_parallel compress profile
set -o pipefail
R=$PWD
for v in old cur old cur; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f64 --mode precision --param 32 --iters 4 --decode 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/r4e_c3_ab.txt
cat gpurun_out/r4e_c3_ab.txt
timeout -k 10 300 python tools/zfp_par_bench.py --reps 3 --profile > gpurun_out/r4e_zpar.txt 2>&1 || exit 1
cat gpurun_out/r4e_zpar.txt
