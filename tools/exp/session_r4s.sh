# round-4 session s: index-scan per-pass trace (4D reversible 128^4, 3D f64 512^3)
set -o pipefail
L=tools/exp/var/trace/libzfp.so
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 > gpurun_out/r4s_scan_trace4.txt 2>&1 || exit 1
ZFP_HIP_SCAN_TRACE=1 ZFP_HIP_SCAN_SEG_BITS=16384 timeout -k 10 200 python tools/scan_bench.py --lib $L --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 > gpurun_out/r4s_scan_trace4_16k.txt 2>&1 || exit 1
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --lib $L --n 512 --reps 1 > gpurun_out/r4s_scan_trace3.txt 2>&1 || exit 1
grep -v "^scan: pass" gpurun_out/r4s_scan_trace4.txt | tail -3
head -20 gpurun_out/r4s_scan_trace4.txt
for v in cur prio cur prio; do
  L=$PWD/tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=
  echo "== $v"
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c4 --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C4', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c3 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C3', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
done > gpurun_out/r4s_prio_ab.txt
cat gpurun_out/r4s_prio_ab.txt
