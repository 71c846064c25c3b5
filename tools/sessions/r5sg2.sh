# index scan: 64 Kbit (default) against 32 Kbit segments, alternating, 4 reps each
mkdir -p gpurun_out
o=gpurun_out/r5sg2_scan_seg_ab.txt
: > $o
for rep in 1 2; do
  for sb in 65536 32768; do
    echo "== rep $rep ZFP_HIP_SCAN_SEG_BITS=$sb" >> $o
    ZFP_HIP_SCAN_SEG_BITS=$sb timeout -k 10 200 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 3 >> $o 2>&1 || exit 1
    ZFP_HIP_SCAN_SEG_BITS=$sb timeout -k 10 200 python tools/scan_bench.py --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 3 >> $o 2>&1 || exit 1
  done
done
