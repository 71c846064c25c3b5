set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_zfpy.py tests/test_zfpy_golden.py tests/test_gpu_distributed.py tests/test_gpu_pipeline.py tests/test_gpu_scan.py -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/zfpy_tests.log 2>&1 || { tail -20 gpurun_out/zfpy_tests.log; exit 1; }
tail -1 gpurun_out/zfpy_tests.log
timeout -k 10 300 python tools/zfp_par_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/zfp_par_bench.py --nparts 16 --threads 16 2>&1 | grep -v amdgpu.ids
