set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in lib lib_var/new4; do
  t=$(echo $v | tr / _)
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_ic_$t -o run -- python $R/tools/kprof.py --iters 2 --decode --lib $R/zfp-par_amd/$v/libzfp.so > $R/gpurun_out/pmc_ic_$t.log 2>&1 || { tail -3 $R/gpurun_out/pmc_ic_$t.log; exit 1; }
  python $R/tools/pmc_table.py $R/gpurun_out/pmc_ic_$t code3 
done
