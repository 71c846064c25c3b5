# A/B: base (before this session) vs current library: 4D decode kernel time, scan parity
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
for v in lib_var/base lib; do
  L=zfp-par_amd/$v/libzfp.so
  echo "== $v"
  $T 120 python tools/kprof.py --lib $L --dims 4 --n 128 --mode reversible --iters 6 --decode 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
  ZFP_HIP_NO_PIPE=1 $T 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  $T 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
