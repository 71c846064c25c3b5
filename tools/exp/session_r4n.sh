# round-4 session n: encoder rare branches laid out cold (variant "ecold") vs product; C3 decoders short vs padded slots
set -o pipefail
for v in cur ecold cur ecold; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --iters 6 2>&1 | grep encode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f64 --mode precision --param 32 --iters 4 2>&1 | grep encode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --mode reversible --iters 4 2>&1 | grep encode || exit 1
done > gpurun_out/r4n_ecold_ab.txt
cat gpurun_out/r4n_ecold_ab.txt
bash tools/exp/session_r4l.sh
