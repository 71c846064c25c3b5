# index scan segment length with plausible starts and refusals: 64 (default), 32, 16, 8 Kbit
mkdir -p gpurun_out
o=gpurun_out/r5sg_scan_seg.txt
: > $o
for sb in 65536 32768 16384 8192; do
  echo "== ZFP_HIP_SCAN_SEG_BITS=$sb" >> $o
  ZFP_HIP_SCAN_SEG_BITS=$sb ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 2 >> $o 2>&1 || exit 1
  ZFP_HIP_SCAN_SEG_BITS=$sb ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 2 >> $o 2>&1 || exit 1
done
