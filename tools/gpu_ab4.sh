set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/pmc_c2stage -o run -- $R/tools/exp/var/c2base c2base stages ) > gpurun_out/pmc_c2stage.log 2>&1 || { tail -5 gpurun_out/pmc_c2stage.log; exit 1; }
python tools/pmc_table.py gpurun_out/pmc_c2stage > gpurun_out/pmc_c2stage.txt; cat gpurun_out/pmc_c2stage.txt
bash tools/ab_lib.sh "--iters 8 --decode" lib lib_var/new4 > gpurun_out/ab4_c2.txt 2>&1 || { tail gpurun_out/ab4_c2.txt; exit 1; }
bash tools/ab_lib.sh "--iters 6 --decode --dtype f64 --mode precision --param 32" lib lib_var/new4 > gpurun_out/ab4_c3.txt 2>&1 || exit 1
bash tools/ab_lib.sh "--iters 6 --decode --mode reversible" lib lib_var/new4 > gpurun_out/ab4_rev.txt 2>&1 || exit 1
grep -h "==\|kernel_ms" gpurun_out/ab4_c2.txt gpurun_out/ab4_c3.txt gpurun_out/ab4_rev.txt
