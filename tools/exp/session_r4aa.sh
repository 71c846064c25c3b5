# round-4 session aa: C5 with the 4D overflow list sorted into block order before the patch pass (variant "osort")
set -o pipefail
L=$PWD/tools/exp/var/osort/libzfp.so
ZFP_BENCH_LIB=$L ZFP_HIP_SLOT_WORDS=15 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_codec4.py > gpurun_out/r4aa_tests.txt 2>&1; tail -1 gpurun_out/r4aa_tests.txt
for v in cur osort cur osort; do
  LL=$PWD/tools/exp/var/$v/libzfp.so; [ $v = cur ] && LL=
  echo "== $v"
  ZFP_BENCH_LIB=$LL timeout -k 10 300 python bench.py --no-cpu --workload c5 --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('C5', d['ms_per_step'], 'ms', d['roofline']['frac'], 'lossless', d.get('lossless_roundtrip'))" || exit 1
done > gpurun_out/r4aa_osort_ab.txt
cat gpurun_out/r4aa_osort_ab.txt
