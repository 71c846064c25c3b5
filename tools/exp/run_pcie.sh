cd $GRAFT_REPO_ROOT
timeout -k 10 120 tools/exp/pcie > gpurun_out/pcie.txt 2>&1; echo rc=$? >> gpurun_out/pcie.txt
bash tools/exp/ab.sh "--iters 6 --mode precision --param 32 --dtype f64" base lb5 > gpurun_out/ab_lb5.txt 2>&1
bash tools/exp/ab.sh "--iters 6 --mode reversible" base lb5 >> gpurun_out/ab_lb5.txt 2>&1
