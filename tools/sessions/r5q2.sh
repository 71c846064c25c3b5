# the reference's array3 on this library; the 4D scan at scale with and without plausible starts
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_arrays.py tests/test_gpu_scan.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5q2_tests.txt 2>&1; echo "tests rc=$?" >> gpurun_out/r5q2_tests.txt
