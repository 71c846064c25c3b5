timeout -k 10 100 ./tools/exp/var/base base > gpurun_out/r4_c2pf4.txt 2>&1
K="python tools/kprof.py --dims 4 --mode reversible --n 128 --iters 8 --decode --sha"
for r in 1 2; do echo "== new"; timeout -k 10 120 $K || exit 1; echo "== w4"; timeout -k 10 120 $K --lib zfp-par_amd/lib_var/e4w4/libzfp.so || exit 1; echo "== e4d4"; timeout -k 10 120 $K --lib zfp-par_amd/lib_var/e4d4/libzfp.so || exit 1; echo "== full slots"; ZFP_HIP_FULL_SLOTS=1 timeout -k 10 120 $K || exit 1; echo "== pack 2117"; ZFP_HIP_PACK_WORDS=2117 timeout -k 10 120 $K || exit 1; done > gpurun_out/r4_4d_ab.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_codec4.py tests/test_gpu_pipeline.py > gpurun_out/r4_t4d.txt 2>&1
