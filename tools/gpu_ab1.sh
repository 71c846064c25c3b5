set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_lib.sh "--iters 8 --decode" lib lib_var/new > gpurun_out/ab1_c2.txt 2>&1 || { tail gpurun_out/ab1_c2.txt; exit 1; }
bash tools/ab_lib.sh "--iters 6 --decode --dtype f64 --mode precision --param 32" lib lib_var/new > gpurun_out/ab1_c3.txt 2>&1 || exit 1
bash tools/ab_lib.sh "--iters 6 --decode --mode reversible" lib lib_var/new > gpurun_out/ab1_rev.txt 2>&1 || exit 1
cat gpurun_out/ab1_*.txt
