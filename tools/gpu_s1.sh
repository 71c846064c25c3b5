# round 3, session 3: parity of the 4D / scan changes, then their timings
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec4.py tests/test_gpu_scan.py \
  tests/test_gpu_pipeline.py tests/test_gpu_types.py tests/test_gpu_golden.py > gpurun_out/s1_tests.log 2>&1 || { tail -30 gpurun_out/s1_tests.log; exit 1; }
tail -2 gpurun_out/s1_tests.log
for A in "--dims 4 --n 128 --mode reversible --iters 6 --decode" "--dims 4 --n 128 --mode rate --param 8 --iters 6 --decode"; do
  echo "== kprof $A"
  $T 120 python tools/kprof.py $A 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
done > gpurun_out/s1_kprof4.txt
cat gpurun_out/s1_kprof4.txt
$T 500 bash tools/exp/scan_lead.sh > gpurun_out/s1_scan_lead.txt 2>&1 || { tail gpurun_out/s1_scan_lead.txt; exit 1; }
cat gpurun_out/s1_scan_lead.txt
$T 300 python bench.py --workload c5 > gpurun_out/s1_bench_c5.json 2> gpurun_out/s1_bench_c5.err || { tail gpurun_out/s1_bench_c5.err; exit 1; }
cat gpurun_out/s1_bench_c5.json
