# round-5 final per-call PMC of C3 and C5 (tools/pmc_bench.sh)
mkdir -p gpurun_out
timeout -k 10 500 bash tools/pmc_bench.sh r5y c3 --sq > gpurun_out/r5y_pmc_c3.log 2>&1 || exit 1
timeout -k 10 600 bash tools/pmc_bench.sh r5y c5 --sq > gpurun_out/r5y_pmc_c5.log 2>&1
