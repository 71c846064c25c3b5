# round-4 session o: 4D reversible encode with short slots (3 waves/SIMD by LDS) and an overflow pool for every block
set -o pipefail
for cfg in "" "ZFP_HIP_SLOT_WORDS=93 ZFP_HIP_OVF_POOL=100000000" "ZFP_HIP_SLOT_WORDS=61 ZFP_HIP_OVF_POOL=100000000" "ZFP_HIP_SLOT_WORDS=45 ZFP_HIP_OVF_POOL=100000000"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/kprof.py --dims 4 --n 128 --mode reversible --iters 5 --sha 2>&1 | grep -E "encode|sha" || exit 1
  env $cfg timeout -k 10 300 python bench.py --no-cpu --workload c5 --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C5', d['ms_per_step'], 'ms', d['roofline']['frac'], 'decode', d.get('decode_ms'), 'lossless', d.get('lossless_roundtrip'))" || exit 1
done > gpurun_out/r4o_4d_slots.txt
cat gpurun_out/r4o_4d_slots.txt
