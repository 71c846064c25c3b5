cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_pipe.txt 2>&1
echo tests=$? >> gpurun_out/t_pipe.txt
tail -3 gpurun_out/t_pipe.txt
grep -q "tests=0" gpurun_out/t_pipe.txt || exit 1
for env in "" "ZFP_HIP_NO_PIPE=1"; do
  echo "== $env" >> gpurun_out/host_pipe.txt
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --param 8 --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --mode precision --param 32 --dtype f64 --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --dims 4 --n 128 --mode reversible --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
done
