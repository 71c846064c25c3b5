set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_lb.txt 2>&1; echo tests=$? >> gpurun_out/t_lb.txt
bash tools/exp/ab.sh "--iters 6 --mode precision --param 32 --dtype f64 --decode" base lb > gpurun_out/ab_lb.txt 2>&1
bash tools/exp/ab.sh "--iters 6 --mode reversible" base lb >> gpurun_out/ab_lb.txt 2>&1
bash tools/exp/ab.sh "--iters 6 --dims 4 --n 128 --mode reversible --decode" base lb >> gpurun_out/ab_lb.txt 2>&1
