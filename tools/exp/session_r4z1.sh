# round-4 final A: the whole GPU suite and the smoke test on the committed build
set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4z_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/r4z_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r4z_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/r4z_smoke.txt 2>&1 || { tail -20 gpurun_out/r4z_smoke.txt; exit 1; }
tail -1 gpurun_out/r4z_smoke.txt
