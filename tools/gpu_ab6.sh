set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/ab_lib.sh "--iters 8 --decode" lib lib_var/thr lib_var/thrA lib_var/thrB > gpurun_out/ab6_c2.txt 2>&1 || { tail gpurun_out/ab6_c2.txt; exit 1; }
bash tools/ab_lib.sh "--iters 6 --decode --dtype f64 --mode precision --param 32" lib lib_var/thr lib_var/thrA lib_var/thrB > gpurun_out/ab6_c3.txt 2>&1 || exit 1
bash tools/ab_lib.sh "--iters 6 --decode --mode reversible" lib lib_var/thr lib_var/thrA lib_var/thrB > gpurun_out/ab6_rev.txt 2>&1 || exit 1
grep -h "==\|kernel_ms" gpurun_out/ab6_c2.txt gpurun_out/ab6_c3.txt gpurun_out/ab6_rev.txt
