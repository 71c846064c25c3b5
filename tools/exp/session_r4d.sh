# round-4 session d: PMC of the 4D reversible kernels on 128^4 and the C3 f64 kernels
set -o pipefail
R=$PWD
timeout -k 10 200 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 --decode --sha > gpurun_out/r4d_4d_time.txt 2>&1 || exit 1
timeout -k 10 200 python tools/kprof.py --dtype f64 --mode precision --param 32 --iters 5 --decode > gpurun_out/r4d_c3_time.txt 2>&1 || exit 1
./tools/pmc_bin.sh r4d_4d -- python $R/tools/kprof.py --dims 4 --n 128 --mode reversible --iters 2 --decode > gpurun_out/r4d_pmc4.log 2>&1 || exit 1
./tools/pmc_bin.sh r4d_c3 -- python $R/tools/kprof.py --dtype f64 --mode precision --param 32 --iters 2 --decode > gpurun_out/r4d_pmc3.log 2>&1 || exit 1
cat gpurun_out/r4d_4d_time.txt gpurun_out/r4d_c3_time.txt
