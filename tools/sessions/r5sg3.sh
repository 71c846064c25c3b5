# product build with 32 Kbit scan segments: GPU scan and codec tests, scan timing
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5sg3_tests.txt 2>&1 || exit 1
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 3 > gpurun_out/r5sg3_scan.txt 2>&1 || exit 1
ZFP_HIP_SCAN_TRACE=1 timeout -k 10 200 python tools/scan_bench.py --n 512 --dims 3 --dtype f64 --mode precision --param 32 --reps 3 >> gpurun_out/r5sg3_scan.txt 2>&1 || exit 1
