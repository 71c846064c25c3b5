# round-4 session r: decode4 group tests from a register window (variant "dwin") vs product
set -o pipefail
for v in cur dwin cur dwin; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --dims 4 --n 128 --mode reversible --iters 5 --decode 2>&1 | grep decode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --dims 4 --n 128 --mode precision --param 20 --iters 5 --decode 2>&1 | grep decode || exit 1
done > gpurun_out/r4r_dwin_ab.txt
cat gpurun_out/r4r_dwin_ab.txt
