# C5 kernel trace: encode4 / fix-ups / encode4_patch / decode4 (packed + overflow) durations
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5v_prof -o run -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/r5v_bench.json 2> $R/gpurun_out/r5v_prof.err || exit 1
cd $R && python tools/prof_tail.py gpurun_out/r5v_prof 20 > gpurun_out/r5v_prof_tail.csv
