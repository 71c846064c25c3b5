set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_ic
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_ic/p1 -o run -- python $R/tools/kprof.py --iters 2 --decode > $R/gpurun_out/pmc_ic/p1.log 2>&1
echo "rc=$?"; tail -3 $R/gpurun_out/pmc_ic/p1.log
