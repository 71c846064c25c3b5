# round-4 session t: priority-1 block loads in encode3_general and encode4 (variant "gprio") vs product
set -o pipefail
for v in cur gprio cur gprio; do
  L=$PWD/tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=
  echo "== $v"
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c3 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C3', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c5 --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C5', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c4 --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C4', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
done > gpurun_out/r4t_gprio_ab.txt
cat gpurun_out/r4t_gprio_ab.txt
