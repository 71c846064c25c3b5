# round 3 final: full GPU suite, smoke, bench (c2) + rocprofv3 trace of it
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3s_gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3s_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3s_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s_smoke.log 2>&1 || { tail gpurun_out/r3s_smoke.log; exit 1; }
tail -1 gpurun_out/r3s_smoke.log
bash tools/round_measure3.sh r3s || exit 1
