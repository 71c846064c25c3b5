# A/B: wave exit in the 32-bit fixed-rate plane loop once every lane's budget is spent (ZFP_FR32_EXIT)
mkdir -p gpurun_out
o=gpurun_out/r5x1.txt
: > $o
bash tools/ab_lib.sh "--param 8 --iters 40 --n 4096 --nz 64 --header" lib lib_var/x16 lib_var/x20 lib_var/x24 >> $o 2>&1 || exit 1
bash tools/ab_lib.sh "--param 16 --iters 40" lib lib_var/x16 lib_var/x24 >> $o 2>&1 || exit 1
