cd $GRAFT_REPO_ROOT
bash tools/exp/ab.sh "--iters 6 --mode precision --param 32 --dtype f64" base lb lb2 lb3 lb4 > gpurun_out/ab_lb2.txt 2>&1
bash tools/exp/ab.sh "--iters 6 --mode reversible" base lb lb2 lb3 lb4 >> gpurun_out/ab_lb2.txt 2>&1
bash tools/exp/ab.sh "--iters 6 --dims 4 --n 128 --mode reversible" base lb lb3 >> gpurun_out/ab_lb2.txt 2>&1
