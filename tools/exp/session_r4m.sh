# round-4 session m: decoder with its rare wave-uniform branches laid out cold (variant "cold") vs product
set -o pipefail
R=$PWD
for v in cur cold cur cold; do
  L=tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=zfp-par_amd/lib/libzfp.so
  echo "== $v"
  timeout -k 10 120 python tools/kprof.py --lib $L --iters 5 --decode 2>&1 | grep decode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --dtype f64 --mode precision --param 32 --iters 4 --decode 2>&1 | grep decode || exit 1
  timeout -k 10 120 python tools/kprof.py --lib $L --mode reversible --iters 4 --decode 2>&1 | grep decode || exit 1
done > gpurun_out/r4m_cold_ab.txt
cat gpurun_out/r4m_cold_ab.txt
cd /tmp && export TMPDIR=/tmp
for v in cur cold; do
  L=$R/tools/exp/var/$v/libzfp.so; [ $v = cur ] && L=$R/zfp-par_amd/lib/libzfp.so
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/r4m_pmc_$v/p1 -o run -- python $R/tools/kprof.py --lib $L --iters 2 --decode > $R/gpurun_out/r4m_pmc_$v.log 2>&1 || exit 1
done
cd $R && python3 tools/pmc_summary.py gpurun_out/r4m_pmc_cur > gpurun_out/r4m_pmc_cur.txt && python3 tools/pmc_summary.py gpurun_out/r4m_pmc_cold > gpurun_out/r4m_pmc_cold.txt; grep -A6 decode3 gpurun_out/r4m_pmc_cur.txt gpurun_out/r4m_pmc_cold.txt
