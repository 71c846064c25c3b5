# per-call HBM traffic of every bench workload (rocprofv3 --pmc, tools/pmc_bench.sh), zfp_parallel loop
mkdir -p gpurun_out
for w in c2 c3 c4 c5; do
  timeout -k 10 400 bash tools/pmc_bench.sh r5h $w --sq > gpurun_out/r5h_pmc_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/zfp_par_bench.py --shape 512 1024 1024 --rate 8 --nparts 8 --threads 8 --reps 3 --loop 6 --profile > gpurun_out/r5h_zpar.txt 2>&1 || exit 1
timeout -k 10 300 python tools/zfp_par_bench.py --shape 512 1024 1024 --precision 20 --nparts 8 --threads 8 --reps 2 --loop 3 > gpurun_out/r5h_zpar_prec.txt 2>&1
