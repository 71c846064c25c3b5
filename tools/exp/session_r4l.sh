# round-4 session l: C3 f64 decoders -- short slots at 3 waves/SIMD (spills) vs padded slots at 2 waves/SIMD (no spills)
set -o pipefail
for cfg in "" "ZFP_HIP_FULL_SLOTS=1" "" "ZFP_HIP_FULL_SLOTS=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/kprof.py --dtype f64 --mode precision --param 32 --iters 4 --decode 2>&1 | grep -E "encode|decode" || exit 1
done > gpurun_out/r4l_c3_slots.txt
cat gpurun_out/r4l_c3_slots.txt
