# round-4 session u: f64 planes-32..63 encoder compiled for 2 waves/SIMD without spills (variant "gw2") vs 3 with 48 B
set -o pipefail
for v in cur gw2 cur gw2; do
  L=$PWD/tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=
  echo "== $v"
  ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --no-cpu --workload c3 --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C3', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'], 'decode', d.get('decode_kernel_ms'))" || exit 1
done > gpurun_out/r4u_gw2_ab.txt
cat gpurun_out/r4u_gw2_ab.txt
