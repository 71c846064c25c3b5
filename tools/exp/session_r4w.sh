# round-4 session w: kernel split of the C5 chunk encode (encode4 vs encode4_patch) from a rocprofv3 trace
set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4w_prof_c5 -o run -- python $R/bench.py --no-cpu --workload c5 --steps 3 --warmup 1 --clock-warm-ms 50 > $R/gpurun_out/r4w_c5.json 2> $R/gpurun_out/r4w_c5.err || exit 1
cd $R
grep -E "encode4|decode4|fixup|Name" gpurun_out/r4w_prof_c5/run_kernel_stats.csv | cut -c1-60,200-330
