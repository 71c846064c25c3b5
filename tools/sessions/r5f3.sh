# bench lines of the product build after the negabinary fold (driver flags): c3, c4, c5
mkdir -p gpurun_out
for w in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/r5f3_bench_$w.json 2> gpurun_out/r5f3_bench_$w.err || exit 1
done
