# round-4 measurement session: GPU suite, bench lines, 4D kernel timings
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r4b_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r4b_gpu_tests.txt
timeout -k 10 300 python bench.py > gpurun_out/r4b_bench_c2.json 2> gpurun_out/r4b_bench_c2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --workload c4 > gpurun_out/r4b_bench_c4.json 2> gpurun_out/r4b_bench_c4.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --workload c5 > gpurun_out/r4b_bench_c5.json 2> gpurun_out/r4b_bench_c5.err || exit 1
timeout -k 10 200 python tools/kprof.py --dims 4 --mode reversible --n 128 --iters 8 --decode --sha > gpurun_out/r4b_kprof4.txt 2>&1 || exit 1
timeout -k 10 200 python tools/zfp_par_bench.py --reps 3 > gpurun_out/r4b_zpar.txt 2>&1 || exit 1
