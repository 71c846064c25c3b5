set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_round.sh r3_old --decode --lib $GRAFT_REPO_ROOT/zfp-par_amd/lib/libzfp.so || exit 1
bash tools/pmc_round.sh r3_new --decode --lib $GRAFT_REPO_ROOT/zfp-par_amd/lib_var/new/libzfp.so || exit 1
python tools/pmc_table.py gpurun_out/pmc_r3_old > gpurun_out/pmc_r3_old.txt
python tools/pmc_table.py gpurun_out/pmc_r3_new > gpurun_out/pmc_r3_new.txt
cat gpurun_out/pmc_r3_old.txt gpurun_out/pmc_r3_new.txt
