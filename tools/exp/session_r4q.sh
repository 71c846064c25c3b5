# round-4 session q: index scan with its window-loop exits marked likely/unlikely (variant "scold") vs product
set -o pipefail
for v in cur scold cur scold; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 200 python tools/scan_bench.py --lib $L --n 512 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/r4q_scan_ab.txt
cat gpurun_out/r4q_scan_ab.txt
