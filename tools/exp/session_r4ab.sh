# round-4 session ab: C2 encoder with LDS-DMA-landed rows (variant "dma") vs product; bit-exactness from the bench's reference leg
set -o pipefail
L=$PWD/tools/exp/var/dma/libzfp.so
ZFP_BENCH_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4ab_dma_c2.json 2>gpurun_out/r4ab_dma_c2.err || { tail -5 gpurun_out/r4ab_dma_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r4ab_dma_c2.json').read().strip().splitlines()[-1]); print('dma', d['roofline']['kernel_ms'], d['roofline']['frac'], 'bitexact', d.get('bitexact_vs_reference'))"
for v in cur dma cur dma; do
  LL=$PWD/tools/exp/var/$v/libzfp.so; [ $v = cur ] && LL=
  ZFP_BENCH_LIB=$LL timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['roofline']['kernel_ms'], 'ms', d['roofline']['frac'])" || exit 1
done
