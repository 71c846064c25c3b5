set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/exp/var/mempat > gpurun_out/ab3_mempat.txt 2>&1 || exit 1
timeout -k 10 120 tools/exp/var/mempat_plain >> gpurun_out/ab3_mempat.txt 2>&1 || exit 1
cat gpurun_out/ab3_mempat.txt
bash tools/ab_lib.sh "--iters 8 --decode" lib lib_var/new3 > gpurun_out/ab3_c2.txt 2>&1 || { tail gpurun_out/ab3_c2.txt; exit 1; }
bash tools/ab_lib.sh "--iters 6 --decode --dtype f64 --mode precision --param 32" lib lib_var/new3 > gpurun_out/ab3_c3.txt 2>&1 || exit 1
bash tools/ab_lib.sh "--iters 6 --decode --mode reversible" lib lib_var/new3 > gpurun_out/ab3_rev.txt 2>&1 || exit 1
grep -h "==\|kernel_ms\|sha" gpurun_out/ab3_c2.txt gpurun_out/ab3_c3.txt gpurun_out/ab3_rev.txt
