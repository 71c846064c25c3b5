set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r3c_tests.log; exit 1; }
tail -3 gpurun_out/r3c_tests.log
for w in c2 c3 c5; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 20 --warmup 10 > gpurun_out/r3c_bench_$w.json 2> gpurun_out/r3c_bench_$w.err || { echo BENCH $w FAILED; tail -20 gpurun_out/r3c_bench_$w.err; exit 1; }
  cat gpurun_out/r3c_bench_$w.json
done
