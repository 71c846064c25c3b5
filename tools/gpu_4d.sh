set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--dims 4 --n 128 --mode reversible --iters 6 --decode"
bash tools/ab_lib.sh "$A" lib lib_var/lbfake > gpurun_out/4d_ab.txt 2>&1 || { tail gpurun_out/4d_ab.txt; exit 1; }
for pw in 1666 2000; do echo "== packw $pw"; ZFP_HIP_VERBOSE=1 ZFP_HIP_PACK_WORDS=$pw timeout -k 10 120 python tools/kprof.py $A 2>&1 | grep -v amdgpu.ids | tail -4; done >> gpurun_out/4d_ab.txt
A8="--dims 4 --n 128 --mode rate --param 8 --iters 6 --decode"
bash tools/ab_lib.sh "$A8" lib >> gpurun_out/4d_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/4d_ab.txt
