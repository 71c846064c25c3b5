mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5i_tests.txt 2>&1; echo "tests rc=$?" >> gpurun_out/r5i_tests.txt
timeout -k 10 200 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/r5i_c5.json 2>&1 || exit 1
timeout -k 10 200 python tools/kprof.py --iters 6 --dims 4 --n 128 --mode reversible --decode > gpurun_out/r5i_k4.txt 2>&1
