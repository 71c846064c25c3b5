# C4 gap: rate 8 on the same 2^30 values with and without the 96-bit header offset, in two geometries
mkdir -p gpurun_out
R=$PWD
o=gpurun_out/r5c4.txt
: > $o
timeout -k 10 120 python tools/kprof.py --param 8 --iters 20 >> $o 2>&1 || exit 1
timeout -k 10 120 python tools/kprof.py --param 8 --iters 20 --header >> $o 2>&1 || exit 1
timeout -k 10 120 python tools/kprof.py --param 8 --iters 20 --n 4096 --nz 64 >> $o 2>&1 || exit 1
timeout -k 10 120 python tools/kprof.py --param 8 --iters 20 --n 4096 --nz 64 --header >> $o 2>&1 || exit 1
timeout -k 10 120 python tools/kprof.py --param 16 --iters 20 --header >> $o 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5c4_prof -o run -- python3 $R/tools/kprof.py --param 8 --iters 20 --n 4096 --nz 64 --header >> $R/$o 2>&1 || exit 1
