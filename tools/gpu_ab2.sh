set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in c2base c2nofru; do timeout -k 10 120 tools/exp/var/$v $v stages || exit 1; done > gpurun_out/ab2_c2var.txt 2>&1
cat gpurun_out/ab2_c2var.txt
bash tools/ab_lib.sh "--iters 8 --decode" lib lib_var/new2 > gpurun_out/ab2_c2.txt 2>&1 || { tail gpurun_out/ab2_c2.txt; exit 1; }
bash tools/ab_lib.sh "--iters 6 --decode --dtype f64 --mode precision --param 32" lib lib_var/new2 > gpurun_out/ab2_c3.txt 2>&1 || exit 1
bash tools/ab_lib.sh "--iters 6 --decode --mode reversible" lib lib_var/new2 > gpurun_out/ab2_rev.txt 2>&1 || exit 1
grep -h "==\|kernel_ms\|sha" gpurun_out/ab2_c2.txt gpurun_out/ab2_c3.txt gpurun_out/ab2_rev.txt
