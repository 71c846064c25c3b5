# round-4 final C: the GPU suite and smoke on the final build, then the C4/C2 bench lines, then the scan counters and C5 split
set -o pipefail
bash tools/exp/session_r4z1.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu --workload c4 > gpurun_out/r4y_bench_c4.json 2> gpurun_out/r4y_bench_c4.err || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r4y_bench_c2.json 2> gpurun_out/r4y_bench_c2.err || exit 1
tail -1 gpurun_out/r4y_bench_c4.json | cut -c1-300
tail -1 gpurun_out/r4y_bench_c2.json | cut -c1-300
bash tools/exp/session_r4v.sh || exit 1
bash tools/exp/session_r4w.sh || exit 1
