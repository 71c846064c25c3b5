# the reference's cfp and array3 on this library
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_arrays.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r5q3_tests.txt 2>&1; echo "tests rc=$?" >> gpurun_out/r5q3_tests.txt
